// Stream-K projection GEMM on the pre-shuffled weight layout:  Y[M,N] = X[M,K] . W[N,K]^T
//
// Why: the 256 x 256 tiles of gemm_big give (M / 256) x (N / 256) tiles, which rarely fill 256 CUs an
// integral number of times -- the headline gate/up projection (M = 512, N = 57344: 448 tiles) runs
// two rounds for 1.75 rounds of work (12.5 % of its time idle), Llama-3-8B prefill gate/up 3.5 rounds.
// Here exactly one persistent workgroup runs per CU and the k-iterations of all tiles are dealt out
// evenly (stream-K), so every CU does the same number of 64-deep k steps:
//
//   * workgroups form GROUPS of mtiles = ceil(M / 256) members, one per 256-row tile, all on one XCD
//     (blocks b, b+8, b+16, ... share an XCD under the dispatcher's round-robin: a placement used for
//     speed only).  A group walks a contiguous range of the (column tile, k step) iteration space; its
//     members compute the same column tile and k range for their own rows at the same time, so every
//     weight tile comes from HBM once and from that XCD's L2 for the other members.
//   * a column tile whose k range is split between groups is finished by the LAST part to arrive: each
//     earlier part takes a ticket, writes its fp32 accumulators (in register order, 1 KB coalesced per
//     wave store) and raises a ready flag (agent-scope release); the last arriver waits for the flags of
//     parts that already hold tickets (resident, never waiting on anything: no deadlock whatever the
//     placement), acquires, sums all parts in fixed group order (deterministic output) and runs the
//     epilogue.  Tickets and flags are reset by the last arriver, so the buffer stays zeroed between
//     launches and graph replays.
//   * the k loop is gemm_big's two-group ping-pong schedule of the 256 x 256 x 64 tile (8 waves, both
//     operands staged by LDS-DMA, 4 phases of 16 MFMA 16x16x32 per stage, row-half 1 one barrier behind,
//     counted vmcnt, raw barriers); epilogues: none / residual add / SiLU(gate) * up.
//
// Reference parity: the q/k/v/o and w1/w2/w3 projections of xotorch/inference/torch/models/
// general_mha.py:77-120 and llm_utils.py:513-522 (torchtune nn.Linear), at serving / prefill batch sizes.
#include "common.h"
#include "gemm_common.h"
#include "kernels.h"

namespace xot {

namespace sk {
constexpr int BM = 256, BN = 256, BK = 64, WM = 2, WN = 4;
constexpr int MT = BM / (16 * WM), NT = BN / (16 * WN);  // 8 x 4 MFMA tiles per wave
constexpr int KS = BK / 32;
constexpr int A_ELEMS = BM * BK, B_ELEMS = BN * BK, STAGE = A_ELEMS + B_ELEMS;
constexpr int A_INSTR = A_ELEMS * 2 / 1024 / 8, B_INSTR = B_ELEMS * 2 / 1024 / 8, NI = A_INSTR + B_INSTR;
constexpr int SMEM = 2 * STAGE * 2;        // two LDS stages: 128 KB
constexpr int PART = BM * BN;              // fp32 elements of one tile's partial accumulators
constexpr int MAX_WG = 256;
}  // namespace sk

// sync words: [0, MAX_WG * 2) ready flags per (workgroup, segment slot); then one ticket per (tile, member)
__device__ __forceinline__ long sk_beg(int g, int G, long total) { return (long)g * total / G; }

// group whose iteration range holds iteration `it`
__device__ __forceinline__ int sk_group_of(long it, int G, long total) {
  int g = (int)((it * G) / total);
  while (g + 1 < G && sk_beg(g + 1, G, total) <= it) ++g;
  while (g > 0 && sk_beg(g, G, total) > it) --g;
  return g;
}

template <int EPI, bool OUT_F32>
__global__ __launch_bounds__(512, 1) void gemm_sk_kernel(const uint16_t* __restrict__ X, int ldx,
                                                         const uint16_t* __restrict__ W,
                                                         const uint16_t* __restrict__ bias,
                                                         const uint16_t* R, int ldr, void* Yv, int ldy,
                                                         float* __restrict__ part, int* __restrict__ sync, int M,
                                                         int N, int K, int mtiles, int gpx) {
  using namespace sk;
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g4 = lane >> 4, c = lane & 15;
  const int wm = wave / WN, wn = wave % WN;

  // ---- group / member of this workgroup (members of a group share an XCD)
  const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
  const int gi = slot / mtiles, member = slot % mtiles;
  if (gi >= gpx) return;  // spare CU of an XCD (32 % mtiles != 0): uniform, before any barrier
  const int G = 8 * gpx, group = xcd * gpx + gi;
  const int ntiles = N / BN, T = K / BK;
  const long total = (long)ntiles * T;
  const long beg = sk_beg(group, G, total), end = sk_beg(group + 1, G, total);
  const int m0 = member * BM, Mv = M;
  int* flags = sync;
  int* tickets = sync + 2 * MAX_WG;

  // ---- per-lane LDS-DMA source offsets (X rows of this member; W offsets relative to the column tile)
  auto aswz = [](int row) -> int { return (row >> 1) & 7; };
  const uint16_t* asrc[A_INSTR];
#pragma unroll
  for (int i = 0; i < A_INSTR; ++i) {
    const int row = 8 * (A_INSTR * wave + i) + lane / 8;
    const int sl = (lane % 8) ^ aswz(row);
    const int grow = min(m0 + row, Mv - 1);  // rows past M load valid memory; their outputs are masked
    asrc[i] = X + (size_t)grow * ldx + sl * 8;
  }
  const int kchunks = K / 128;
  // W: instruction i of this wave copies 1 KB block (i % KS) of 16-row group 2 * wave + i / KS; only lane * 8
  // varies over the lanes (the rest is wave-uniform, kept in scalar registers)
  static_assert(B_INSTR == 2 * KS, "two 16-row groups per wave per stage");
  const size_t wgrp = (size_t)(B_INSTR / KS) * wave * kchunks * 2048;
  // A fragments: rows wm * 128 + 16 i + c; the slot swizzle (row >> 1) & 7 = (c >> 1) & 7 does not depend on
  // i, so the offsets of row slice i are those of slice 0 plus a constant
  int aoff0[KS];
#pragma unroll
  for (int s2 = 0; s2 < KS; ++s2) {
    const int row = wm * (MT * 16) + c;
    aoff0[s2] = row * BK + (((4 * s2 + g4) ^ aswz(row)) * 8);
  }
  const int boff = (wn * NT) * KS * 512 + lane * 8;

  auto bar = []() {  // raw barrier (no vmcnt / lgkmcnt drain); the asm statements are compiler fences
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  const int half = __builtin_amdgcn_readfirstlane(wm);

  f32x4 acc[MT][NT];
  for (long it = beg; it < end;) {
    const int tile = (int)(it / T), kb = (int)(it % T);
    const int ke = (int)min((long)T, kb + (end - it));
    it += ke - kb;
    const uint16_t* Wt = W + (size_t)(tile * (BN / 16)) * kchunks * 2048;

#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    auto issue = [&](int t, int buf) {  // k step t -> LDS buffer buf
      uint16_t* As = smem + buf * STAGE;
      uint16_t* Bs = As + A_ELEMS;
      const int k0 = t * BK;
      const size_t woff = (size_t)(k0 >> 7) * 2048 + ((k0 & 127) >> 5) * 512;
#pragma unroll
      for (int i = 0; i < A_INSTR; ++i) glds16<0>(asrc[i] + k0, As + (A_INSTR * wave + i) * 512);
#pragma unroll
      for (int i = 0; i < B_INSTR; ++i)
        glds16<3>(Wt + wgrp + (size_t)(i / KS) * kchunks * 2048 + (i % KS) * 512 + woff + lane * 8,
                  Bs + (B_INSTR * wave + i) * 512);
    };
    s16x8 af[4][2], bq[2][2][2];
    auto read_a = [&](int buf, int qm) {
      const uint16_t* As = smem + buf * STAGE;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) af[i][s2] = ld16(As + aoff0[s2] + (4 * qm + i) * 16 * BK);
    };
    auto read_b = [&](int buf, int qn) {
      const uint16_t* Bs = smem + buf * STAGE + A_ELEMS;
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) bq[qn][j][s2] = ld16(Bs + boff + ((2 * qn + j) * KS + s2) * 512);
    };
    auto quad = [&](int qm, int qn) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[4 * qm + i][2 * qn + j] = mfma16(af[i][s2], bq[qn][j][s2], acc[4 * qm + i][2 * qn + j]);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
    };

    const int Tn = ke - kb;  // >= 1
    issue(kb, 0);
    if (Tn > 1) {
      issue(kb + 1, 1);
      wait_vm<NI>();
    } else {
      wait_vm<0>();
    }
    bar();
    if (half == 1) bar();  // row-half 1 runs one barrier behind
    for (int t = 0; t < Tn; ++t) {
      const int buf = t & 1;
      read_a(buf, 0);  // phase 0
      read_b(buf, 0);
      bar();
      quad(0, 0);
      bar();
      read_b(buf, 1);  // phase 1 (last B read of this stage)
      bar();
      quad(0, 1);
      bar();
      read_a(buf, 1);  // phase 2 (last A read of this stage)
      bar();
      quad(1, 1);
      bar();
      // phase 3: every wave finished reading this buffer -> refill it with stage t+2; retire stage t+1
      if (t + 2 < Tn) {
        issue(kb + t + 2, buf);
        wait_vm<NI>();
      } else {
        wait_vm<0>();
      }
      bar();
      quad(1, 0);
      bar();
    }
    if (half == 0) bar();  // balance the barrier count
    __syncthreads();       // all LDS reads of this segment done (no LDS-DMA in flight: vmcnt(0) above)

    // ---- stream-K fixup: which groups share this column tile?
    int g_first = sk_group_of((long)tile * T, G, total);
    int g_last = sk_group_of((long)tile * T + T - 1, G, total);
    bool last = true;
    if (g_first != g_last) {
      int* sh = reinterpret_cast<int*>(smem);
      const int tk = tile * mtiles + member;
      if (tid == 0) sh[0] = __hip_atomic_fetch_add(&tickets[tk], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __syncthreads();
      const int ticket = sh[0];
      last = ticket == g_last - g_first;
      // segment slot of (group, tile): 0 = the group's first tile, 1 = its last
      auto slot_of = [&](int g) { return (tile == (int)(sk_beg(g, G, total) / T)) ? 0 : 1; };
      auto part_of = [&](int g) {
        return part + ((size_t)((g * mtiles + member) * 2 + slot_of(g))) * PART + (size_t)wave * (MT * NT * 256);
      };
      auto flag_of = [&](int g) { return &flags[(g * mtiles + member) * 2 + slot_of(g)]; };
      if (!last) {
        float* p = part_of(group);
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
          for (int j = 0; j < NT; ++j) *reinterpret_cast<f32x4*>(p + ((i * NT + j) * 64 + lane) * 4) = acc[i][j];
        wait_vm<0>();
        __syncthreads();
        if (tid == 0) {
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          // 0 -> 1 publishes; -1 means the last arriver gave up on this part (timed out, tile poisoned):
          // consume that mark back to 0, so a late publish never leaves a stale 1 for the next launch (stream
          // order guarantees this wave finishes before the next launch of the stream starts)
          int expect = 0;
          if (!__hip_atomic_compare_exchange_strong(flag_of(group), &expect, 1, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT))
            __hip_atomic_store(flag_of(group), 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      } else {
        if (tid == 0) {
          int stale = 0;
          for (int g = g_first; g <= g_last; ++g) {
            if (g == group) continue;
            int* f = flag_of(g);
            // bounded: a part that holds a ticket is resident and publishes within microseconds; the bound
            // (seconds) only keeps a broken invariant from hanging the GPU
            int spin = 0;
            for (; spin < (1 << 24) && __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 1; ++spin)
              __builtin_amdgcn_s_sleep(2);
            if (spin == (1 << 24)) {
              // timed out: mark the part abandoned (-1) unless it published in the meantime (then clear it)
              stale = 1;
              int expect = 0;
              if (!__hip_atomic_compare_exchange_strong(f, &expect, -1, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT))
                __hip_atomic_store(f, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
              __hip_atomic_store(f, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
          }
          __hip_atomic_store(&tickets[tk], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          sh[1] = stale;
        }
        __syncthreads();
        if (sh[1]) {
          // a peer part never published (broken invariant): poison the tile with NaN so the failure shows
          // in every consumer instead of passing a sum over stale / unwritten partials
#pragma unroll
          for (int i = 0; i < MT; ++i)
#pragma unroll
            for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{__builtin_nanf(""), __builtin_nanf(""), __builtin_nanf(""), __builtin_nanf("")};
          g_last = group;  // skip the summation below
          g_first = group;
        }
        // sum the parts in group order (own accumulators at this group's position: deterministic output),
        // one 16-row slice of the wave's tile at a time (each part's 4 loads per lane in flight together)
#pragma unroll
        for (int i = 0; i < MT; ++i) {
          f32x4 t[NT], u[NT];
          bool have = false;
          for (int g = g_first; g < group; ++g) {
            const float* p = part_of(g) + (i * NT * 64 + lane) * 4;
#pragma unroll
            for (int j = 0; j < NT; ++j) u[j] = *reinterpret_cast<const f32x4*>(p + j * 256);
#pragma unroll
            for (int j = 0; j < NT; ++j) t[j] = have ? t[j] + u[j] : u[j];
            have = true;
          }
          if (have) {
#pragma unroll
            for (int j = 0; j < NT; ++j) acc[i][j] = t[j] + acc[i][j];
          }
          for (int g = group + 1; g <= g_last; ++g) {
            const float* p = part_of(g) + (i * NT * 64 + lane) * 4;
#pragma unroll
            for (int j = 0; j < NT; ++j) u[j] = *reinterpret_cast<const f32x4*>(p + j * 256);
#pragma unroll
            for (int j = 0; j < NT; ++j) acc[i][j] += u[j];
          }
        }
      }
    }
    if (!last) continue;

    // ---- epilogue of column tile `tile`, rows m0 ..
    // (row strides laundered through an empty asm: otherwise the 32 per-row output offsets are hoisted out of
    // the tile loop and held in 64 VGPRs across the k loop -- spilled to scratch at 256 VGPRs)
    int ldy_e = ldy, ldr_e = ldr;
    asm volatile("" : "+s"(ldy_e), "+s"(ldr_e));
    const int rbase = m0 + wm * (MT * 16);
    const int cbase = tile * BN + wn * (NT * 16);
    if constexpr (EPI == EPI_SILU) {
#pragma unroll
      for (int p = 0; p < NT / 2; ++p) {  // (gate tile 2p, up tile 2p+1) -> 16 output columns
        const int col = (cbase >> 1) + 16 * p + c;
        float bg = 0.f, bu = 0.f;
        if (bias != nullptr) {
          bg = bf2f(bias[cbase + 32 * p + c]);
          bu = bf2f(bias[cbase + 32 * p + 16 + c]);
        }
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int m = rbase + 16 * i + 4 * g4 + r;
            if (m < Mv) {
              const float v = silu(acc[i][2 * p][r] + bg) * (acc[i][2 * p + 1][r] + bu);
              if constexpr (OUT_F32)
                reinterpret_cast<float*>(Yv)[(size_t)m * ldy_e + col] = v;
              else
                reinterpret_cast<uint16_t*>(Yv)[(size_t)m * ldy_e + col] = f2bf(v);
            }
          }
      }
    } else {
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int col = cbase + 16 * j + c;
        const float bv = bias != nullptr ? bf2f(bias[col]) : 0.f;
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int m = rbase + 16 * i + 4 * g4 + r;
            if (m < Mv) {
              float v = acc[i][j][r] + bv;
              if constexpr (EPI == EPI_RESID) v += bf2f(R[(size_t)m * ldr_e + col]);
              if constexpr (OUT_F32)
                reinterpret_cast<float*>(Yv)[(size_t)m * ldy_e + col] = v;
              else
                reinterpret_cast<uint16_t*>(Yv)[(size_t)m * ldy_e + col] = f2bf(v);
            }
          }
      }
    }
  }
}

// workspace sizes (elements) the caller provides: partial fp32 slots and zeroed int sync words
long gemm_sk_part_elems() { return (long)sk::MAX_WG * 2 * sk::PART; }
long gemm_sk_sync_words(int M, int N) { return 2L * sk::MAX_WG + (long)((M + 255) / 256) * (N / 256); }

template <int EPI, bool F32>
static void sk_launch(const uint16_t* X, int ldx, const uint16_t* W, const uint16_t* bias, const uint16_t* R, int ldr,
                      void* Y, int ldy, float* part, int* sync, int M, int N, int K, int mtiles, int gpx, int cus,
                      hipStream_t st) {
  auto kern = gemm_sk_kernel<EPI, F32>;
  static bool attr =
      hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, sk::SMEM) == hipSuccess;
  (void)attr;
  kern<<<cus, 512, sk::SMEM, st>>>(X, ldx, W, bias, R, ldr, Y, ldy, part, sync, M, N, K, mtiles, gpx);
}

// cus: workgroups to launch (one per CU, a multiple of 8, at most 256)
int launch_gemm_sk(const uint16_t* X, int ldx, const uint16_t* W, const uint16_t* bias, const uint16_t* R, int ldr,
                   void* Y, int ldy, bool out_f32, int epi, float* part, int* sync, int M, int N, int K, int cus,
                   hipStream_t s) {
  if (M <= 0) return 0;
  if (N % 256 != 0 || K % 128 != 0 || cus % 8 != 0 || cus <= 0 || cus > sk::MAX_WG) return -1;
  if (epi == EPI_SILU && N % 32 != 0) return -1;
  const int mtiles = (M + 255) / 256;
  const int per_xcd = cus / 8;
  if (mtiles > per_xcd) return -1;  // a group must fit one XCD's share of the CUs
  const int gpx = per_xcd / mtiles;
  // every group needs a non-empty k range (a column tile's parts are the groups between its first and last)
  if ((long)(N / 256) * (K / 64) < 8L * gpx) return -1;
  if (epi == EPI_SILU) {
    if (out_f32) sk_launch<EPI_SILU, true>(X, ldx, W, bias, R, ldr, Y, ldy, part, sync, M, N, K, mtiles, gpx, cus, s);
    else sk_launch<EPI_SILU, false>(X, ldx, W, bias, R, ldr, Y, ldy, part, sync, M, N, K, mtiles, gpx, cus, s);
  } else if (epi == EPI_RESID) {
    if (out_f32) return -1;
    sk_launch<EPI_RESID, false>(X, ldx, W, bias, R, ldr, Y, ldy, part, sync, M, N, K, mtiles, gpx, cus, s);
  } else {
    if (out_f32) sk_launch<EPI_NONE, true>(X, ldx, W, bias, R, ldr, Y, ldy, part, sync, M, N, K, mtiles, gpx, cus, s);
    else sk_launch<EPI_NONE, false>(X, ldx, W, bias, R, ldr, Y, ldy, part, sync, M, N, K, mtiles, gpx, cus, s);
  }
  return 0;
}

}  // namespace xot

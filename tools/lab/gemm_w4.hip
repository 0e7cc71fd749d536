// LAB (not shipped; measured slower than gemm_big's ping-pong at every shape, at the same power cap:
// profiles/r4/lab4/).  Four-wave 256 x 256 GEMM on the pre-shuffled weight layout:  Y[M,N] = X[M,K] . W[N,K]^T
//
// Why a second large-M kernel: at M >= 512 every GEMM of this library runs at the board's power cap
// (profiles/r4/power/), so what sets its rate is the energy per FLOP.  gemm_big's eight waves own 128 x 64 of
// the tile each and read 24 KB of LDS fragments per wave per 64-deep k step (192 KB per CU); four waves of
// 128 x 128 read 32 KB each (128 KB per CU, -33 %) for the same FLOPs, the shape the vendor library picks for
// tall GEMMs.  The price is one wave per SIMD (256 fp32 accumulators + two fragment sets per lane), so the
// schedule must hide the LDS and memory latency inside ONE wave's instruction stream:
//   * k stages of 32 (32 KB: X 256 x 32 and W 256 x 32), NB buffers; a stage's fragments move to registers one
//     stage ahead, so its buffer is refilled (stage t + NB) right after the barrier of stage t: NB - 1 stages in
//     flight under the MFMAs (LDS-DMA issued by every wave: 4 X + 4 W 1-KB instructions per stage)
//   * the fragments of stage t + 1 (8 A + 8 B ds_read_b128 per wave) are read while the 64 MFMAs of stage t
//     run, in 8 groups of 8 MFMAs (sched_barrier between groups): group q consumes A fragment q against all 8
//     B fragments, so A fragment q of stage t + 1 is read into the same registers right after it, and B
//     fragment q into the second B set -- 96 fragment registers instead of 128, no spill beside the 256
//     accumulators; one LDS-DMA pair per two groups
//   * per stage: vmcnt retires stage t + 1 (leaving the younger ones in flight), lgkmcnt(0) retires this
//     wave's reads of stage t, the barrier then frees stage t's buffer for every wave and publishes stage
//     t + 1 (cdna_hip_programming.md "Pipelining across barriers": raw s_barrier, counted vmcnt)
// X tile [256 rows][32 k] in LDS with 64-B rows, 16-B slots XOR-swizzled per 4-row group (the gemm_big BK = 32
// map, applied through the LDS-DMA source address); W tile = 16 row groups x one 1-KB k32 block each.
// Tile order, split-K slabs and epilogues as gemm_big.  Reference parity: the projections of
// xotorch/inference/torch/models/llm_utils.py:513-522 / general_mha.py:77-120 (torchtune nn.Linear).
#include "../../xotorch_support_jetson_amd/csrc/common.h"
#include "../../xotorch_support_jetson_amd/csrc/gemm_common.h"

#include <type_traits>

namespace xot {

namespace w4 {
constexpr int BM = 256, BN = 256, BK = 32;
// acc += a . b with the accumulator pinned in place in AGPRs: with 256 accumulators per lane the compiler's
// own MFMA form renames them between loop iterations and shuffles them through VGPRs (v_accvgpr moves and
// scratch spills); the tied "+a" operand keeps each in one AGPR quad for the whole k loop.
__device__ __forceinline__ void mfma_acc(f32x4& acc, const s16x8& a, const s16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}
constexpr int A_ELEMS = BM * BK, STAGE = (BM + BN) * BK;  // bf16 elements per stage (32 KB)
template <int NB>
constexpr int smem() { return NB * STAGE * 2; }
}  // namespace w4

template <int EPI, bool OUT_F32, bool SPLIT, int NB, int ILV = 0>
__global__ __launch_bounds__(256, 1) void gemm_w4_kernel(const uint16_t* __restrict__ X, int ldx,
                                                         const uint16_t* __restrict__ W,
                                                         const uint16_t* __restrict__ bias,
                                                         const uint16_t* __restrict__ R, int ldr,
                                                         void* __restrict__ Yv, int ldy, float* __restrict__ ws,
                                                         int M, int N, int K, int S) {
  using namespace w4;
  static_assert(NB >= 3 && NB <= 5, "3..5 stage buffers (<= 160 KB)");
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c = lane & 15;
  const int wm = wave >> 1, wn = wave & 1;

  // ---- tile: bijective XCD remap, then split-major; tall grids in groups of 4 row tiles (gemm_big's order)
  const int mtiles = (M + BM - 1) / BM, ntiles = (N + BN - 1) / BN;
  const int nwg = mtiles * ntiles * S;
  int b = blockIdx.x;
  {
    const int xcd = b & 7, q = nwg >> 3, r = nwg & 7;
    b = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
  }
  int mt, nt, split;
  {
    constexpr int GROUP_M = 4;
    const int tiles = mtiles * ntiles;
    split = b / tiles;
    const int bt = b - split * tiles;
    if (mtiles >= 2 * GROUP_M) {
      const int per = GROUP_M * ntiles, grp = bt / per, first = grp * GROUP_M;
      const int gm = min(mtiles - first, GROUP_M), rr = bt - grp * per;
      mt = first + rr % gm;
      nt = rr / gm;
    } else {
      mt = bt % mtiles;
      nt = bt / mtiles;
    }
  }
  const int m0 = mt * BM, n0 = nt * BN;
  const int T_all = K / BK;
  const int t_beg = (int)((long)split * T_all / S), t_end = (int)((long)(split + 1) * T_all / S);
  const int T = t_end - t_beg;

  // X: 64-B rows, slot (row >> 2)-swizzled {0, 2, 3, 1}
  auto aswz = [](int row) -> int {
    constexpr int lut = 0 | (2 << 2) | (3 << 4) | (1 << 6);
    return (lut >> (2 * ((row >> 2) & 3))) & 3;
  };
  // LDS-DMA sources: X instruction i (16 rows: 4 lanes per row) = 4 * wave + i; W instruction i = row group
  // 4 * wave + i of the tile (its 1-KB k32 block)
  const uint16_t* asrc[4];
  const uint16_t* bsrc[4];
  const size_t kchunks = K / 128;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = 16 * (4 * wave + i) + (lane >> 2);
    const int slot = (lane & 3) ^ aswz(row);
    asrc[i] = X + (size_t)min(m0 + row, M - 1) * ldx + slot * 8;  // rows past M re-read the last; outputs masked
    const int grp = min((n0 >> 4) + 4 * wave + i, N / 16 - 1);
    bsrc[i] = W + (size_t)grp * kchunks * 2048 + lane * 8;
  }
  auto issue = [&](int t, int buf, int i) {  // LDS-DMA pair i (one X + one W instruction) of stage t
    uint16_t* As = smem + buf * STAGE;
    const int k0 = (t_beg + t) * BK;
    glds16<0>(asrc[i] + k0, As + (4 * wave + i) * 512);
    glds16<3>(bsrc[i] + (size_t)(k0 >> 7) * 2048 + ((k0 & 127) >> 5) * 512, As + A_ELEMS + (4 * wave + i) * 512);
  };

  // fragment offsets (elements) inside a stage
  int aoff[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int row = wm * 128 + 16 * i + c;
    aoff[i] = row * BK + ((g ^ aswz(row)) * 8);
  }
  const int boff = A_ELEMS + (wn * 8) * 512 + lane * 8;  // + j * 512

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  s16x8 fa[8], fb[2][8];
  auto read_a = [&](int buf, int q) { fa[q] = ld16(smem + buf * STAGE + aoff[q]); };
  auto read_b = [&](int buf, int set, int q) { fb[set][q] = ld16(smem + buf * STAGE + boff + q * 512); };
  auto bar = []() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  if (T > 0) {
    // prologue: stages 0 .. NB-1 in flight; stage 0 landed; its fragments into set 0
#pragma unroll
    for (int p = 0; p < NB; ++p) {
#pragma unroll
      for (int i = 0; i < 4; ++i) issue(min(p, T - 1), p, i);  // past the end: the last stage again (unused)
    }
    wait_vm<8 * (NB - 1)>();
    bar();
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      read_a(0, q);
      read_b(0, 0, q);
    }

    // one k stage; SET = B register set holding stage t's fragments (compile-time: the loop is unrolled by 2).
    // The body is the same for every stage: past the end of the k range the refill re-loads the last stage
    // into the buffer just freed (never read again) and the read-ahead reads a stale buffer (never used), so
    // the loop has no branches between its MFMA groups and the in-flight count is always NB - 1 stages.
    auto stage = [&](int t, auto set_c) {
      constexpr int SET = decltype(set_c)::value;
      wait_vm<8 * (NB - 2)>();  // stage t+1 landed (this wave's DMA); its younger stages stay in flight
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // stage t's fragments are in registers
      bar();  // stage t+1 landed for every wave; stage t's buffer free for every wave
      const int rbuf = t % NB, nbuf = (t + 1) % NB;
      const int tr = min(t + NB, T - 1);
      // 64 MFMAs in 8 groups of 8; after group q: A fragment q and B fragment q of stage t+1, and (q even)
      // one LDS-DMA pair of stage t + NB
#pragma unroll
      for (int q = 0; q < 8; ++q) {
#pragma unroll
        for (int j = 0; j < 8; ++j) mfma_acc(acc[q][j], fa[q], fb[SET][j]);
        read_a(nbuf, q);
        read_b(nbuf, SET ^ 1, q);
        if ((q & 1) == 0) issue(tr, rbuf, q >> 1);
        if constexpr (ILV == 0) {
          __builtin_amdgcn_sched_barrier(0);
        } else {
          // one wave per SIMD hides single-issue work only BETWEEN its MFMAs: spread the group's LDS reads,
          // DMA issue and address arithmetic over its 8 MFMAs instead of bunching them after the last one
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // one MFMA
            if (u == 1 || u == 5) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // one DS read
            if ((u == 3 || u == 7) && (q & 1) == 0) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // one VMEM
            __builtin_amdgcn_sched_group_barrier(0x006, 2, 0);  // up to two VALU / SALU
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    };
    int t = 0;
    for (; t + 1 < T; t += 2) {
      stage(t, std::integral_constant<int, 0>{});
      stage(t + 1, std::integral_constant<int, 1>{});
    }
    if (t < T) stage(t, std::integral_constant<int, 0>{});
    wait_vm<0>();
  }

  // the last MFMAs (inline asm: invisible to the hazard recognizer) retire before any VALU reads their results
  asm volatile("s_nop 7\n s_nop 7\n s_nop 7" ::: "memory");
  // ---- epilogue (lane (g, c): rows 16 i + 4 g + r, column 16 j + c of the wave's 128 x 128)
  const int rbase = m0 + wm * 128, cbase = n0 + wn * 128;
  if constexpr (SPLIT) {
    float* slab = ws + (size_t)split * M * N;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = rbase + 16 * i + 4 * g + r;
        if (m < M) {
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (cbase + 16 * j < N) slab[(size_t)m * N + cbase + 16 * j + c] = acc[i][j][r];
        }
      }
  } else if constexpr (EPI == EPI_SILU) {
#pragma unroll
    for (int p = 0; p < 4; ++p) {  // (gate tile 2p, up tile 2p+1) -> 16 output columns
      const int gcol = cbase + 32 * p;
      if (gcol >= N) break;
      const int col = (gcol >> 1) + c;
      float bg = 0.f, bu = 0.f;
      if (bias != nullptr) {
        bg = bf2f(bias[gcol + c]);
        bu = bf2f(bias[gcol + 16 + c]);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = rbase + 16 * i + 4 * g + r;
          if (m < M) {
            const float v = silu(acc[i][2 * p][r] + bg) * (acc[i][2 * p + 1][r] + bu);
            if constexpr (OUT_F32)
              reinterpret_cast<float*>(Yv)[(size_t)m * ldy + col] = v;
            else
              reinterpret_cast<uint16_t*>(Yv)[(size_t)m * ldy + col] = f2bf(v);
          }
        }
    }
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (cbase + 16 * j >= N) break;
      const int col = cbase + 16 * j + c;
      const float bv = bias != nullptr ? bf2f(bias[col]) : 0.f;
#pragma unroll
      for (int i0 = 0; i0 < 8; i0 += 4) {
        float rv[4][4];
        if constexpr (EPI == EPI_RESID) {
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              rv[i][r] = bf2f(R[(size_t)min(rbase + 16 * (i0 + i) + 4 * g + r, M - 1) * ldr + col]);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int m = rbase + 16 * (i0 + i) + 4 * g + r;
            if (m < M) {
              float v = acc[i0 + i][j][r] + bv;
              if constexpr (EPI == EPI_RESID) v += rv[i][r];
              if constexpr (OUT_F32)
                reinterpret_cast<float*>(Yv)[(size_t)m * ldy + col] = v;
              else
                reinterpret_cast<uint16_t*>(Yv)[(size_t)m * ldy + col] = f2bf(v);
            }
          }
      }
    }
  }
}

}  // namespace xot

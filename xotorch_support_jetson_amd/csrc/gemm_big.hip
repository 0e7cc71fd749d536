// Large-M projection GEMM on the pre-shuffled weight layout:  Y[M,N] = X[M,K] . W[N,K]^T
//
// Serves decode batches above 128 rows and prefill chunks -- the compute-bound regime, where the
// weight-streaming kernel (gemm.hip) runs out of MFMA issue rate.  Structure (CDNA4, wave64):
//   * workgroup tile 256 (M) x BN (N) x 64 (K), 8 waves (512 threads) as WM x WN; a wave owns
//     (256/WM) x (BN/WN) of the output = MT x NT tiles of v_mfma_f32_16x16x32_bf16
//   * both operands staged HBM/L2 -> LDS by LDS-DMA (global_load_lds_dwordx4, 1 KB per wave
//     instruction, no VGRP round trip), two stages: stage t+1 is issued before the MFMAs of stage t
//     and retired by one counted wait + one barrier per 64-deep k step
//   * W tiles: the shuffled layout stores the MFMA B fragments of 16 rows x 32 k as 1 KB, so a
//     16-row group's 64-deep stage is 2 KB of contiguous memory copied verbatim; fragment reads are
//     ds_read_b128 at lane*16 (conflict-free)
//   * X tiles: [256 rows][64 k] with 128-B rows; 16-B slot XOR-swizzled by (row >> 1) & 7 (applied
//     to the per-lane global source address, so the LDS-DMA image stays lane-linear) -> the 16-lane
//     groups of every A-fragment ds_read_b128 hit 16 distinct bank quads
//   * XCD-aware block order: consecutive tile ids (the row tiles of one column tile, then the next
//     column tiles) are dispatched to the same XCD, so a weight tile is read from HBM once and the
//     activation rows stay in that XCD's L2
//   * fused epilogues (bias, residual add, SiLU(gate)*up on 16-row interleaved gate/up weights) or
//     split-K fp32 slabs reduced by splitk_reduce_kernel
//
// Reference parity: the q/k/v/o and w1/w2/w3 projections of xotorch/inference/torch/models/
// general_mha.py:77-120 and llm_utils.py:513-522 (torchtune nn.Linear), at serving batch sizes.
#include "common.h"
#include "gemm_common.h"
#include "kernels.h"

namespace xot {


// AUXA / AUXB: cache-policy bits of the X / W LDS-DMA loads (sc0 = 1, nt = 2, sc1 = 16)
// MOE = 1 / 2: grouped GEMM over experts (blockIdx.y = expert e, weight W[e], rows moe_off[e] ..
// moe_off[e+1] of the expert-sorted slot order; MOE 2 gathers X row moe_gather[slot]); M is the
// worst-case rows per expert (row tiles past an expert's count exit at once, so the grid is fixed and
// graph-capturable).  A K split writes fp32 partial slabs ysplit elements apart (summed by the consumer).
// MOE = 4: K-grouped GEMM (the weight gradients of grouped experts): blockIdx.y = group e multiplies the k
// range [moe_off[e], moe_off[e+1]) (multiples of BK) of the shared operands X [M, K] and W [N, K] into
// Y_e = Y + e M ldy (and R_e for the residual epilogue); an empty range stores bias / residual only.
// PP: two-group ping-pong schedule (BM = BN = 256, 2 x 4 waves, BK = 64, 2 buffers): each 64-deep stage
// is 4 phases of 16 MFMAs (one 64 x 32 quadrant of the wave's 128 x 64 tile); phase = {fragment reads ->
// barrier -> MFMAs -> barrier}; the row-half-1 waves run one barrier behind, so on every SIMD one wave's
// MFMAs overlap the other's LDS reads.  A stage is read only in its phases 0-2 (A halves in 0 and 2, B
// halves in 0 and 1), so in phase 3 the stage two ahead is issued into the buffer being finished, and
// the stage one ahead is retired by a counted vmcnt (LDS-DMA stays in flight across the barriers).
// (Schedules measured slower and removed: an 8-phase per-half refill and a three-deep weight pipeline,
// profiles/r3/lab_gemm_schedules_random.log, profiles/r3/lab_s2/w_three_deep_staging.log; 512 x 128 tiles,
// profiles/r4/lab3.)
template <int BM, int BN, int WM, int WN, int BK, int NBUF, int EPI, bool OUT_F32, bool SPLIT, int MOE = 0, int AUXA = 0,
          int AUXB = 3, int PP = 0>
__global__ __launch_bounds__(512, 1) void gemm_big_kernel(const uint16_t* __restrict__ X, int ldx,
                                                          const uint16_t* __restrict__ W,
                                                          const uint16_t* __restrict__ bias,
                                                          const uint16_t* __restrict__ R, int ldr,
                                                          void* __restrict__ Yv, int ldy, float* __restrict__ ws,
                                                          int M, int N, int K, int S,
                                                          const int* __restrict__ moe_off = nullptr,
                                                          const int* __restrict__ moe_gather = nullptr,
                                                          long ysplit = 0, int group_m = 4) {
  static_assert(WM * WN == 8, "8 waves");
  static_assert(BK == 32 || BK == 64, "k stage of 32 or 64");
  static_assert(BM % (16 * WM) == 0 && BM >= 128 && BM <= 512, "row tile of 128 .. 512 rows");
  static_assert(PP == 0 || PP == 1 || PP == 2, "schedules: base (0), ping-pong in 4 phases (1) or 2 phases (2)");
  static_assert(MOE == 0 || MOE == 4 || (!SPLIT && EPI != EPI_RESID), "grouped GEMM: no slab reduce, no residual");
  static_assert(MOE != 4 || !SPLIT, "K-grouped GEMM: no K split");
  constexpr int MT = BM / (16 * WM), NT = BN / (16 * WN);
  // odd NT (BN = 224: 7 row groups per wave): the gate/up pair that straddles two waves of a row is
  // joined through LDS in the epilogue
  static_assert(EPI != EPI_SILU || NT % 2 == 0 || (PP == 0 && MOE == 0), "SiLU epilogue pairs gate/up n-tiles");
  constexpr int KS = BK / 32;                          // MFMA k-steps (and 1 KB W blocks per row group) per stage
  constexpr int SPR = BK / 8;                          // 16-B slots per X row in LDS
  constexpr int A_ELEMS = BM * BK, B_ELEMS = BN * BK;  // bf16 elements per stage
  constexpr int STAGE = A_ELEMS + B_ELEMS;
  // 1 KB LDS-DMA instructions per stage: NAI (X) and NBI (W) in all, A_INSTR / B_INSTR per wave.  When a
  // count is not a multiple of 8 (BM = 224: 28 X instructions; BN = 224: 28 W instructions) the waves below
  // count % 8 issue one more than the others (instruction q = 8 i + wave) and each wave retires its own count.
  constexpr int NAI = A_ELEMS * 2 / 1024, NBI = B_ELEMS * 2 / 1024;
  constexpr int A_INSTR = (NAI + 7) / 8, B_INSTR = (NBI + 7) / 8;
  constexpr bool A_UNEVEN = NAI % 8 != 0, B_UNEVEN = NBI % 8 != 0;
  static_assert(!(A_UNEVEN || B_UNEVEN) || PP == 0, "uneven instruction split: base schedule only");
  constexpr int NI = A_INSTR + B_INSTR;
  constexpr int PD = NBUF - 1;                         // stages in flight ahead of the one computed
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c = lane & 15;
  const int wm = wave / WN, wn = wave % WN;

  // ---- tile of this workgroup (bijective XCD remap, then split-major / column / row order, grouped when tall)
  const int mtiles = (M + BM - 1) / BM, ntiles = (N + BN - 1) / BN;  // N % BN != 0: a masked last column tile
  const int nwg = mtiles * ntiles * S;
  int b = blockIdx.x;
  {
    const int xcd = b & 7, q = nwg >> 3, r = nwg & 7;
    b = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
  }
  // Tall grids (prefill, training: 8+ row tiles) are rastered in groups of group_m row tiles x every column tile,
  // column-major inside a group: the ~32 workgroups an XCD runs at once then cover 4 row tiles x 8 column tiles
  // (12 distinct operand slices per k step in its L2) instead of one column tile x 32 row tiles (33).  Short
  // grids (decode: 1-2 row tiles) keep the plain row-fastest order, which is already that.
  // (group_m: 4 by default, XOT_GEMM_GROUP_M; <= 1 keeps the row-fastest order)
  int mt, nt, split;
  {
    const int tiles = mtiles * ntiles;
    split = b / tiles;
    const int bt = b - split * tiles;
    if ((MOE == 0 || MOE == 4) && group_m > 1 && mtiles >= 2 * group_m) {
      const int per = group_m * ntiles, grp = bt / per, first = grp * group_m;
      const int gm = min(mtiles - first, group_m), rr = bt - grp * per;
      mt = first + rr % gm;
      nt = rr / gm;
    } else {
      mt = bt % mtiles;
      nt = bt / mtiles;
    }
  }
  const int m0 = mt * BM, n0 = nt * BN;
  int row0 = 0, Mv = M;  // first output row (slot) and valid rows of this launch's row range
  if constexpr (MOE == 1 || MOE == 2) {
    const int e = blockIdx.y;
    row0 = moe_off[e];
    Mv = moe_off[e + 1] - row0;
    W += (size_t)e * N * K;
    if (m0 >= Mv) return;  // uniform over the workgroup, before any barrier
    if (ysplit != 0) Yv = reinterpret_cast<float*>(Yv) + (size_t)split * ysplit;
  }
  const int T_all = K / BK;
  int t_beg = (int)((long)split * T_all / S), t_end = (int)((long)(split + 1) * T_all / S);
  if constexpr (MOE == 4) {
    const int e = blockIdx.y;
    t_beg = moe_off[e] / BK;
    t_end = moe_off[e + 1] / BK;
    if constexpr (OUT_F32)
      Yv = reinterpret_cast<float*>(Yv) + (size_t)e * M * ldy;
    else
      Yv = reinterpret_cast<uint16_t*>(Yv) + (size_t)e * M * ldy;
    if (R != nullptr) R += (size_t)e * M * ldr;
  }
  const int T = t_end - t_beg;

  // X LDS image: rows of BK bf16, 16-B slot XOR-swizzled so the 16 lanes of each A-fragment
  // ds_read_b128 group land on 16 distinct bank quads (2 rows per 256-B bank row at BK = 64, 4 at 32).
  auto aswz = [](int row) -> int {
    if constexpr (SPR == 8) {
      return (row >> 1) & 7;
    } else {
      constexpr int lut = 0 | (2 << 2) | (3 << 4) | (1 << 6);  // {0, 2, 3, 1}
      return (lut >> (2 * ((row >> 2) & 3))) & 3;
    }
  };

  // ---- LDS-DMA source addresses (advance with the k stage)
  // X: instruction i of wave w covers rows (1024 / (2*BK)) * (A_INSTR*w + i) .. ; lane -> row +lane/SPR,
  // physical slot lane%SPR holding logical slot (lane%SPR) ^ aswz(row).
  const uint16_t* asrc[A_INSTR];
  auto aq = [&](int i) { return A_UNEVEN ? 8 * i + wave : A_INSTR * wave + i; };
#pragma unroll
  for (int i = 0; i < A_INSTR; ++i) {
    const int row = (64 / SPR) * min(aq(i), NAI - 1) + lane / SPR;
    const int slot = (lane % SPR) ^ aswz(row);
    int grow = min(m0 + row, Mv - 1);  // rows past the end load valid memory; their outputs are masked
    if constexpr (MOE == 1) grow += row0;
    if constexpr (MOE == 2) grow = moe_gather[row0 + grow];
    asrc[i] = X + (size_t)grow * ldx + slot * 8;
  }
  // W: instruction q = B_INSTR*w + i copies 1 KB block q % KS of row group q / KS for this stage.
  const size_t kchunks = K / 128;
  const uint16_t* bsrc[B_INSTR];
  auto bq = [&](int i) { return B_UNEVEN ? 8 * i + wave : B_INSTR * wave + i; };
#pragma unroll
  for (int i = 0; i < B_INSTR; ++i) {
    const int q = min(bq(i), NBI - 1);
    const int grp = min((n0 >> 4) + q / KS, N / 16 - 1);  // groups past N re-read the last one; outputs masked
    bsrc[i] = W + ((size_t)grp * kchunks) * 2048 + (q % KS) * 512 + lane * 8;
  }
  // this wave's LDS-DMA instructions per stage (wave-uniform)
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  const int ni_w = NI - (A_UNEVEN && wave_u >= NAI % 8 ? 1 : 0) - (B_UNEVEN && wave_u >= NBI % 8 ? 1 : 0);

  auto issue = [&](int t, int buf) {  // stage t (absolute k step) -> LDS buffer buf
    uint16_t* As = smem + buf * STAGE;
    uint16_t* Bs = As + A_ELEMS;
    const int k0 = t * BK;
    const size_t woff = (size_t)(k0 >> 7) * 2048 + ((k0 & 127) >> 5) * 512;
#pragma unroll
    for (int i = 0; i < A_INSTR; ++i)
      if (!A_UNEVEN || aq(i) < NAI) glds16<AUXA>(asrc[i] + k0, As + aq(i) * 512);
#pragma unroll
    for (int i = 0; i < B_INSTR; ++i)
      if (!B_UNEVEN || bq(i) < NBI) glds16<AUXB>(bsrc[i] + woff, Bs + bq(i) * 512);
  };

  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment read offsets (elements) inside a stage
  int aoff[MT][KS];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int row = wm * (MT * 16) + 16 * i + c;
#pragma unroll
    for (int s2 = 0; s2 < KS; ++s2) aoff[i][s2] = row * BK + (((4 * s2 + g) ^ aswz(row)) * 8);
  }
  const int boff = (wn * NT) * KS * 512 + lane * 8;  // + (16-row group j)*KS*512 + s2*512

  // Per stage: B fragments of all k-steps first, then the A fragments in a ring LDPF deep so each
  // ds_read_b128 is in flight under the MFMAs of the previous row tile (the scheduling fence keeps
  // the compiler from hoisting all reads up front, which costs registers and serialises on lgkmcnt).
  constexpr int LDPF = 3;
  auto compute_ab = [&](const uint16_t* As, const uint16_t* Bs) {
    s16x8 bf[KS][NT];
#pragma unroll
    for (int s2 = 0; s2 < KS; ++s2)
#pragma unroll
      for (int j = 0; j < NT; ++j) bf[s2][j] = ld16(Bs + boff + (j * KS + s2) * 512);
    s16x8 af[LDPF];
#pragma unroll
    for (int u = 0; u < LDPF; ++u) af[u] = ld16(As + aoff[u % MT][u / MT]);
#pragma unroll
    for (int u = 0; u < KS * MT; ++u) {
      const int s2 = u / MT, i = u % MT;
      const s16x8 cur = af[u % LDPF];
      if (u + LDPF < KS * MT) af[u % LDPF] = ld16(As + aoff[(u + LDPF) % MT][(u + LDPF) / MT]);
#pragma unroll
      for (int j = 0; j < NT; ++j) acc[i][j] = mfma16(cur, bf[s2][j], acc[i][j]);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  auto compute = [&](int buf) { compute_ab(smem + buf * STAGE, smem + buf * STAGE + A_ELEMS); };

  // Barrier without the vmcnt(0) drain __syncthreads() would add: LDS-DMA stages stay in flight.
  // The asm statements are compiler fences (no LDS access moves across the barrier).
  auto barrier = []() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  // wait until at most k younger stages of this wave are still in flight
  auto wait_stages = [&](int k) {
    if constexpr (!A_UNEVEN && !B_UNEVEN) {
      if (PD >= 4 && k >= 3) wait_vm<(PD >= 4 ? 3 * NI : 0)>();
      else if (PD >= 3 && k >= 2) wait_vm<(PD >= 3 ? 2 * NI : 0)>();
      else if (PD >= 2 && k >= 1) wait_vm<(PD >= 2 ? NI : 0)>();
      else wait_vm<0>();
    } else {
      wait_vm_upto<(PD - 1) * NI>(max(0, min(k, PD - 1)) * ni_w);
    }
  };

  if constexpr (PP == 1 || PP == 2) {
    static_assert((BM == 256 || BM == 192 || BM == 128) && BN == 256 && WM == 2 && WN == 4 && BK == 64 && NBUF == 2, "PP geometry");
    constexpr int MQ = MT / 2;  // row tiles per A half of a wave (4 at BM 256, 3 at BM 192)
    auto bar = []() {  // raw barrier (no vmcnt / lgkmcnt drain); the asm statements are compiler fences
      asm volatile("" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    };
    s16x8 af[MQ][2], bq[2][2][2];
    auto read_a = [&](int buf, int qm) {
      const uint16_t* As = smem + buf * STAGE;
#pragma unroll
      for (int i = 0; i < MQ; ++i)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) af[i][s2] = ld16(As + aoff[MQ * qm + i][s2]);
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
        for (int i = 0; i < MQ; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[MQ * qm + i][2 * qn + j] = mfma16(af[i][s2], bq[qn][j][s2], acc[MQ * qm + i][2 * qn + j]);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
    };
    if (T > 0) {
      issue(t_beg, 0);
      if (T > 1) {
        issue(t_beg + 1, 1);
        wait_vm<NI>();
      } else {
        wait_vm<0>();
      }
      bar();
      // wave-uniform branch (an EXEC-masked s_barrier would still execute)
      const int half = __builtin_amdgcn_readfirstlane(wm);
      if (half == 1) bar();  // row-half 1 runs one barrier behind
      if constexpr (PP == 2) {
      for (int t = 0; t < T; ++t) {
        // two phases of 32 MFMAs: {A half 0, both B halves} -> quads (0,0), (0,1); {A half 1, refill with stage
        // t+2, retire stage t+1} -> quads (1,1), (1,0).  Four barriers per stage instead of eight.
        const int buf = t & 1;
        read_a(buf, 0);
        read_b(buf, 0);
        read_b(buf, 1);
        bar();
        quad(0, 0);
        quad(0, 1);
        bar();
        read_a(buf, 1);  // last read of this stage by this wave
        // Refill with stage t+2 here, in the read phase: a wave's LDS-DMA issue inside its MFMA phase costs more
        // than the whole schedule gains (measured: refill after the barrier, or only the A rows the group is
        // still reading moved there, ran slower than the four-phase schedule, profiles/r4/pp2/).  The refill
        // lands >= one L2 round trip after issue, while the reads it could overtake -- the group's own A rows
        // here, issued at the start of this phase, and the other group's B reads, issued before the previous
        // barrier -- complete within one LDS round trip (the same margin the four-phase schedule relies on).
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (t + 2 < T) {
          issue(t_beg + t + 2, buf);
          wait_vm<NI>();
        } else {
          wait_vm<0>();
        }
        bar();
        quad(1, 1);
        quad(1, 0);
        bar();
      }
      } else {
      for (int t = 0; t < T; ++t) {
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
        // phase 3: every wave finished reading this buffer two barriers ago -> refill it with stage t+2;
        // retire stage t+1 (the younger stage t+2 stays in flight)
        if (t + 2 < T) {
          issue(t_beg + t + 2, buf);
          wait_vm<NI>();
        } else {
          wait_vm<0>();
        }
        bar();
        quad(1, 0);
        bar();
      }
      }
      if (half == 0) bar();  // balance the barrier count
    }
  } else if (T > 0) {
    // prologue: stages 0 .. PD-1 in flight, stage 0 landed
#pragma unroll
    for (int p = 0; p < PD; ++p)
      if (p < T) issue(t_beg + p, p);
    wait_stages(min(PD - 1, T - 1));
    barrier();
    for (int t = 0; t < T; ++t) {
      // refill the buffer computed in iteration t-1 (every wave is past that iteration's barrier)
      if (t + PD < T) issue(t_beg + t + PD, (t + PD) % NBUF);
      compute(t % NBUF);
      // stage t+1 landed for this wave; the barrier makes it landed for all
      wait_stages(min(PD - 1, T - 2 - t));
      barrier();
    }
  }

  // ---- epilogue
  const int rbase = m0 + wm * (MT * 16);
  if constexpr (MOE == 1 || MOE == 2) {  // output rows are slots
    if constexpr (OUT_F32)
      Yv = reinterpret_cast<float*>(Yv) + (size_t)row0 * ldy;
    else
      Yv = reinterpret_cast<uint16_t*>(Yv) + (size_t)row0 * ldy;
  }
  const int cbase = n0 + wn * (NT * 16);
  if constexpr (SPLIT) {
    float* slab = ws + (size_t)split * M * N;
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = rbase + 16 * i + 4 * g + r;
        if (m < Mv) {
#pragma unroll
          for (int j = 0; j < NT; ++j)
            if (cbase + 16 * j < N) slab[(size_t)m * N + cbase + 16 * j + c] = acc[i][j][r];
        }
      }
  } else if constexpr (EPI == EPI_SILU) {
    // (gate group at column gcol, up group at gcol + 16) -> 16 output columns starting at gcol / 2
    auto store_pair = [&](int gcol, auto gate, auto up) {
      if (gcol >= N) return;
      const int col = (gcol >> 1) + c;
      float bg = 0.f, bu = 0.f;
      if (bias != nullptr) {
        bg = bf2f(bias[gcol + c]);
        bu = bf2f(bias[gcol + 16 + c]);
      }
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = rbase + 16 * i + 4 * g + r;
          if (m < Mv) {
            const float v = silu(gate(i)[r] + bg) * (up(i)[r] + bu);
            if constexpr (OUT_F32)
              reinterpret_cast<float*>(Yv)[(size_t)m * ldy + col] = v;
            else
              reinterpret_cast<uint16_t*>(Yv)[(size_t)m * ldy + col] = f2bf(v);
          }
        }
    };
    if constexpr (NT % 2 == 0) {
#pragma unroll
      for (int p = 0; p < NT / 2; ++p)  // (gate tile 2p, up tile 2p+1)
        store_pair(cbase + 32 * p, [&](int i) { return acc[i][2 * p]; }, [&](int i) { return acc[i][2 * p + 1]; });
    } else {
      // odd NT, 2 wave columns: wave column 0 holds pairs (0,1) .. and the GATE of the straddling pair in
      // its last tile; wave column 1 holds that pair's UP in its tile 0, then pairs (1,2) ..  The up tile
      // crosses through LDS (the stage buffers are idle: the k loop ended on a drained barrier).
      static_assert(WN == 2 && MOE == 0 && !SPLIT, "odd NT: two wave columns, plain GEMM");
      float* xch = reinterpret_cast<float*>(smem);
      const int wcol = __builtin_amdgcn_readfirstlane(wn);
      if (wcol == 1) {
#pragma unroll
        for (int i = 0; i < MT; ++i) *reinterpret_cast<f32x4*>(xch + ((wm * MT + i) * 64 + lane) * 4) = acc[i][0];
      }
      barrier();
      if (wcol == 0) {
#pragma unroll
        for (int p = 0; p < NT / 2; ++p)
          store_pair(cbase + 32 * p, [&](int i) { return acc[i][2 * p]; }, [&](int i) { return acc[i][2 * p + 1]; });
        store_pair(cbase + 16 * (NT - 1), [&](int i) { return acc[i][NT - 1]; },
                   [&](int i) { return *reinterpret_cast<const f32x4*>(xch + ((wm * MT + i) * 64 + lane) * 4); });
      } else {
#pragma unroll
        for (int p = 0; p < NT / 2; ++p)
          store_pair(cbase + 16 + 32 * p, [&](int i) { return acc[i][1 + 2 * p]; },
                     [&](int i) { return acc[i][2 + 2 * p]; });
      }
    }
  } else {
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      if (cbase + 16 * j >= N) break;
      const int col = cbase + 16 * j + c;
      const float bv = bias != nullptr ? bf2f(bias[col]) : 0.f;
      // residuals of this column tile loaded up front (one latency for MT x 4 loads; the per-element
      // load-add-store chain exposed it per element: +50 % on accumulating dW GEMMs); rows past Mv
      // re-read row Mv - 1 and are not stored.  In place (R == Y) is safe: each element is read and
      // written by this lane only.
      constexpr int IP = MT >= 4 ? MT / 2 : MT;  // row tiles per prefetch group (register budget)
#pragma unroll
      for (int i0 = 0; i0 < MT; i0 += IP) {
      float rv[IP][4];
      if constexpr (EPI == EPI_RESID) {
#pragma unroll
        for (int i = 0; i < IP; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            rv[i][r] = bf2f(R[(size_t)min(rbase + 16 * (i0 + i) + 4 * g + r, Mv - 1) * ldr + col]);
      }
#pragma unroll
      for (int i = 0; i < IP; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = rbase + 16 * (i0 + i) + 4 * g + r;
          if (m < Mv) {
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

template <int BM, int BN, int BK, int NBUF>
constexpr int big_smem() {  // LDS bytes of a gemm_big configuration
  return NBUF * (BM + BN) * BK * 2;
}

// grouped raster width of tall plain grids (XOT_GEMM_GROUP_M, read once; default 4)
int gemm_big_group_m();
static int big_group_m() { return gemm_big_group_m(); }
int gemm_big_group_m() {
  static const int gm = [] {
    const char* e = getenv("XOT_GEMM_GROUP_M");
    return e != nullptr ? atoi(e) : 4;
  }();
  return gm;
}

template <int BM, int BN, int WM, int WN, int BK, int NBUF, int EPI, bool F32, int PP = 0>
static void big_launch(const uint16_t* X, int ldx, const uint16_t* W, const uint16_t* bias, const uint16_t* R,
                       int ldr, void* Y, int ldy, float* ws, int M, int N, int K, int S, bool reduce,
                       hipStream_t st) {
  constexpr int SMEM = big_smem<BM, BN, BK, NBUF>();
  static_assert(SMEM <= 160 * 1024, "LDS");
  const int nwg = ((M + BM - 1) / BM) * ((N + BN - 1) / BN) * S;
  if (S == 1) {
    auto kern = gemm_big_kernel<BM, BN, WM, WN, BK, NBUF, EPI, F32, false, 0, 0, 3, PP>;
    static bool attr = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM) ==
                       hipSuccess;
    (void)attr;
    kern<<<nwg, 512, SMEM, st>>>(X, ldx, W, bias, R, ldr, Y, ldy, nullptr, M, N, K, 1, nullptr, nullptr, 0L,
                                 big_group_m());
  } else {
    auto kern = gemm_big_kernel<BM, BN, WM, WN, BK, NBUF, EPI, false, true, 0, 0, 3, PP>;
    static bool attr = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM) ==
                       hipSuccess;
    (void)attr;
    kern<<<nwg, 512, SMEM, st>>>(X, ldx, W, bias, R, ldr, Y, ldy, ws, M, N, K, S, nullptr, nullptr, 0L,
                                 big_group_m());
    if (!reduce) return;  // slabs left for the consumer (fused reduce + residual + RMSNorm)
    const int ncol = EPI == EPI_SILU ? N / 2 : N;
    const long chunks = (long)M * (ncol / 8);
    int blocks = (int)((chunks + 255) / 256);
    if (blocks > 2048) blocks = 2048;
    splitk_reduce_kernel<EPI, F32><<<blocks, 256, 0, st>>>(ws, S, M, N, bias, R, ldr, Y, ldy);
  }
}

template <int EPI, bool F32>
static int big_dispatch(const uint16_t* X, int ldx, const uint16_t* W, const uint16_t* bias, const uint16_t* R,
                        int ldr, void* Y, int ldy, float* ws, long ws_elems, int M, int N, int K, int bn, int S,
                        bool reduce, hipStream_t st) {
  // bn = tile code: BN (256 / 128 / 224), 1256 / 2256 (256 x 256 on the four- / two-phase ping-pong), plus
  // 10000 x BM for row tiles below 256 (160 / 192 / 224: M = 320 / 384 / 448 in two tiles without padding rows;
  // 2256 only with 192)
  const int bm = bn / 10000 ? bn / 10000 : 256, code = bn % 10000;
  if (code == 4256 && bm == 256) {  // four-wave 256 x 256 tile (gemm_w4.hip)
    const int rc = launch_gemm_w4(X, ldx, W, bias, R, ldr, Y, ldy, F32, EPI, ws, M, N, K, S, big_group_m(), st);
    if (rc != 0 || S == 1 || !reduce) return rc;
    const int ncol = EPI == EPI_SILU ? N / 2 : N;
    const long chunks = (long)M * (ncol / 8);
    int blocks = (int)((chunks + 255) / 256);
    if (blocks > 2048) blocks = 2048;
    splitk_reduce_kernel<EPI, F32><<<blocks, 256, 0, st>>>(ws, S, M, N, bias, R, ldr, Y, ldy);
    return 0;
  }
#define XOT_BIG(BM_, BN_, WM_, NBUF_, ...)                                                                        \
  big_launch<BM_, BN_, WM_, 8 / WM_, 64, NBUF_, EPI, F32, ##__VA_ARGS__>(X, ldx, W, bias, R, ldr, Y, ldy, ws, M, N, K, \
                                                                         S, reduce, st)
  if (bm == 256) {
    if (code == 256) XOT_BIG(256, 256, 2, 2);
    else if (code == 1256) XOT_BIG(256, 256, 2, 2, 1);  // ping-pong schedule of the 256 x 256 tile
    else if (code == 2256) XOT_BIG(256, 256, 2, 2, 2);  // the same in two phases per stage (4 barriers, not 8)
    else if (code == 128) XOT_BIG(256, 128, 4, 3);
    else if (code == 224) XOT_BIG(256, 224, 4, 2);      // 7 row groups per wave (gate/up N = 57344 -> 256 tiles)
    else return -1;
  } else if (code == 256) {
    if (bm == 224) XOT_BIG(224, 256, 2, 2);
    else if (bm == 192) XOT_BIG(192, 256, 2, 2);
    else if (bm == 160) XOT_BIG(160, 256, 2, 2);
    else return -1;
  } else if (code == 2256) {
    if (bm == 192) XOT_BIG(192, 256, 2, 2, 2);  // two-phase ping-pong on 192-row tiles (three row tiles per A half)
    else return -1;
  } else if (code == 128) {
    if (bm == 224) XOT_BIG(224, 128, 2, 3);
    else if (bm == 192) XOT_BIG(192, 128, 2, 3);
    else if (bm == 160) XOT_BIG(160, 128, 2, 3);
    else return -1;
  } else {
    return -1;
  }
#undef XOT_BIG
  return 0;
}

int launch_gemm_big(const uint16_t* X, int ldx, const uint16_t* W, const uint16_t* bias, const uint16_t* R, int ldr,
                    void* Y, int ldy, bool out_f32, int epi, float* ws, long ws_elems, int M, int N, int K, int bn,
                    int S, bool reduce, hipStream_t s) {
  if (M <= 0) return 0;
  if (N % 16 != 0 || K % 128 != 0 || S < 1 || S > K / 64) return -1;  // tile codes: big_dispatch
  if (S > 1 && (ws == nullptr || ws_elems < (long)S * M * N)) return -1;
  if (epi == EPI_SILU && N % 32 != 0) return -1;
  if (epi == EPI_SILU)
    return out_f32 ? big_dispatch<EPI_SILU, true>(X, ldx, W, bias, R, ldr, Y, ldy, ws, ws_elems, M, N, K, bn, S, reduce, s)
                   : big_dispatch<EPI_SILU, false>(X, ldx, W, bias, R, ldr, Y, ldy, ws, ws_elems, M, N, K, bn, S, reduce, s);
  if (epi == EPI_RESID)
    return out_f32 ? -1 : big_dispatch<EPI_RESID, false>(X, ldx, W, bias, R, ldr, Y, ldy, ws, ws_elems, M, N, K, bn, S, reduce, s);
  return out_f32 ? big_dispatch<EPI_NONE, true>(X, ldx, W, bias, R, ldr, Y, ldy, ws, ws_elems, M, N, K, bn, S, reduce, s)
                 : big_dispatch<EPI_NONE, false>(X, ldx, W, bias, R, ldr, Y, ldy, ws, ws_elems, M, N, K, bn, S, reduce, s);
}

// ------------------------------------------------------------------------------------ K-grouped (expert dW)
// Y_e [M, N] (+)= X[:, koff[e]:koff[e+1]] . W[:, koff[e]:koff[e+1]]^T for e < E; X [M, K] row-major, W [N, K]
// pre-shuffled, koff multiples of 64 (segments padded with zero rows by the caller), resid: Y_e += (in place).
int launch_gemm_kgroup(const uint16_t* X, int ldx, const uint16_t* W, uint16_t* Y, int ldy, bool resid,
                       const int* koff, int E, int M, int N, int K, hipStream_t st) {
  if (M <= 0 || E <= 0 || N <= 0) return 0;
  if (N % 16 != 0 || K % 128 != 0) return -1;
  constexpr int SMEM = 2 * (256 + 256) * 64 * 2;
  const dim3 grid(((M + 255) / 256) * ((N + 255) / 256), E);
  if (resid) {
    auto kern = gemm_big_kernel<256, 256, 2, 4, 64, 2, EPI_RESID, false, false, 4, 0, 3, 2>;
    static bool attr = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM) ==
                       hipSuccess;
    (void)attr;
    kern<<<grid, 512, SMEM, st>>>(X, ldx, W, nullptr, Y, ldy, Y, ldy, nullptr, M, N, K, 1, koff, nullptr, 0L,
                                  big_group_m());
  } else {
    auto kern = gemm_big_kernel<256, 256, 2, 4, 64, 2, EPI_NONE, false, false, 4, 0, 3, 2>;
    static bool attr = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM) ==
                       hipSuccess;
    (void)attr;
    kern<<<grid, 512, SMEM, st>>>(X, ldx, W, nullptr, nullptr, 0, Y, ldy, nullptr, M, N, K, 1, koff, nullptr, 0L,
                                  big_group_m());
  }
  return 0;
}

// S fp32 slabs [S][M][N] of a 16-row interleaved gate/up product -> silu(gate) * up [M, N/2] bf16
void launch_splitk_silu(const float* ws, int S, int M, int N, uint16_t* y, hipStream_t s) {
  if (M <= 0) return;
  const long chunks = (long)M * (N / 2 / 8);
  int blocks = (int)((chunks + 255) / 256);
  if (blocks > 2048) blocks = 2048;
  splitk_reduce_kernel<EPI_SILU, false><<<blocks, 256, 0, s>>>(ws, S, M, N, nullptr, nullptr, 0, y, N / 2);
}

// ------------------------------------------------------------------------------------ grouped (MoE)
template <int BM, int EPI, bool F32, int MOE, int BK = 64, int NBUF = 2, int PP = 0>
static void big_moe_launch(const uint16_t* X, int ldx, const uint16_t* W, void* Y, int ldy, const int* off,
                           const int* gather, int E, int max_rows, int N, int K, int S, long ysplit, hipStream_t st) {
  constexpr int BN = 256, WM = 2, WN = 4;
  constexpr int SMEM = NBUF * (BM + BN) * BK * 2;
  static_assert(SMEM <= 160 * 1024, "LDS");
  auto kern = gemm_big_kernel<BM, BN, WM, WN, BK, NBUF, EPI, F32, false, MOE, 0, 3, PP>;
  static bool attr = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM) ==
                     hipSuccess;
  (void)attr;
  dim3 grid(((max_rows + BM - 1) / BM) * (N / BN) * S, E);
  kern<<<grid, 512, SMEM, st>>>(X, ldx, W, nullptr, nullptr, 0, Y, ldy, nullptr, max_rows, N, K, S, off, gather,
                                S > 1 ? ysplit : 0L, 4);
}

// bm = row tile (128 / 192 / 256) + 1000 x pipeline variant: 0 = two 64-deep LDS stages (one in flight under
// the MFMAs); 1 = more expert-weight bytes in flight for the HBM-bound groups (BM 128: three 64-deep stages;
// BM 192 / 256: four 32-deep stages, three in flight); 2 (BM 192 / 256) = the two-phase ping-pong schedule
template <int EPI, bool F32>
static void big_moe_bm(const uint16_t* X, int ldx, const uint16_t* W, void* Y, int ldy, const int* off,
                       const int* gather, int E, int max_rows, int N, int K, int S, long ysplit, int bm,
                       hipStream_t st) {
#define XOT_MOE(BM_, ...)                                                                                          \
  do {                                                                                                            \
    if (gather)                                                                                                   \
      big_moe_launch<BM_, EPI, F32, 2, ##__VA_ARGS__>(X, ldx, W, Y, ldy, off, gather, E, max_rows, N, K, S, ysplit, st); \
    else                                                                                                          \
      big_moe_launch<BM_, EPI, F32, 1, ##__VA_ARGS__>(X, ldx, W, Y, ldy, off, gather, E, max_rows, N, K, S, ysplit, st); \
  } while (0)
  switch (bm) {
    case 128: XOT_MOE(128); break;
    case 192: XOT_MOE(192); break;
    case 1128: XOT_MOE(128, 64, 3); break;
    case 1192: XOT_MOE(192, 32, 4); break;
    case 1256: XOT_MOE(256, 32, 4); break;
    case 2256: XOT_MOE(256, 64, 2, 2); break;  // 256- / 192-row tiles on the two-phase ping-pong schedule
    case 2192: XOT_MOE(192, 64, 2, 2); break;
    case 2128: XOT_MOE(128, 64, 2, 2); break;
    default: XOT_MOE(256); break;
  }
#undef XOT_MOE
}

int launch_gemm_moe_big(const uint16_t* X, int ldx, const uint16_t* W, void* Y, int ldy, bool out_f32, int epi,
                        const int* off, const int* gather, int E, int max_rows, int N, int K, int S, long ysplit,
                        int bm, hipStream_t s) {
  if (max_rows <= 0) return 0;
  if ((bm % 1000 != 128 && bm % 1000 != 192 && bm % 1000 != 256) || (bm > 1256 && bm != 2256 && bm != 2192 && bm != 2128) || N % 256 != 0 ||
      K % 128 != 0 || S < 1 ||
      S > K / 64)
    return -1;
  if (epi != EPI_NONE && epi != EPI_SILU) return -1;
  if (epi == EPI_SILU && out_f32) return -1;
  if (S > 1 && (epi != EPI_NONE || !out_f32)) return -1;  // K slices write fp32 partial slabs
  if (epi == EPI_SILU)
    big_moe_bm<EPI_SILU, false>(X, ldx, W, Y, ldy, off, gather, E, max_rows, N, K, S, ysplit, bm, s);
  else if (out_f32)
    big_moe_bm<EPI_NONE, true>(X, ldx, W, Y, ldy, off, gather, E, max_rows, N, K, S, ysplit, bm, s);
  else
    big_moe_bm<EPI_NONE, false>(X, ldx, W, Y, ldy, off, gather, E, max_rows, N, K, S, ysplit, bm, s);
  return 0;
}

}  // namespace xot

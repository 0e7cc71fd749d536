// Four-wave 256 x 256 x 64 GEMM on the pre-shuffled weight layout (tile code 4256):  Y[M,N] = X[M,K] . W[N,K]^T
//
// The large-M shapes of prefill and training (M >= 1024: a dozen k stages or more per tile) run gemm_big's
// eight-wave ping-pong at ~1.55 us per 64-deep k step and 18 us of fixed cost per tile; hipBLASLt's
// MT256x256x64 kernel takes ~1.33 us and 11 us (profiles/r5/gemm_overhead/).  This kernel follows the
// schedule that gets there (one wave per SIMD, everything of a stage in registers early):
//   * 4 waves, each 128 x 128 of the tile: 64 accumulator tiles (256 AGPRs) and ALL 32 fragments of a
//     64-deep stage in registers (128 VGPRs) -- 0.25 fragment reads per MFMA instead of 0.375
//   * two LDS stage buffers (2 x 64 KB, LDS-DMA, 16 1-KB instructions per wave and stage); a stage's buffer is
//     free as soon as every wave holds its fragments, so stage t+2 is issued a quarter into stage t and has
//     ~1.5 stages of latency budget (the ping-pong tile's refill has ~1)
//   * per stage: half 0's 64 MFMAs with half 1's 16 fragment reads under the first 16; lgkmcnt(0) + barrier after
//     32; 16 LDS-DMA issues spread over the next 64 MFMAs; vmcnt + barrier (stage t+1 landed); stage t+1's half-0
//     fragments read under MFMAs 32..47 of half 1, in the order the MFMAs consume them -- two barriers per 128
//     MFMAs, every fragment read 16 MFMAs ahead of its first use
// Operand roles are swapped against gemm_big: the MFMA A operand is the weight fragment (16 output columns x 32 k),
// B the activation fragment (32 k x 16 tokens), so a lane's accumulator holds 4 consecutive output COLUMNS of one
// token.  With PERM (every epilogue but SiLU) the weight rows of each pair of 16-column tiles are read permuted
// (tile 2J row m = column 32 J + 8 (m >> 2) + (m & 3) + 4 (j & 1)), so a lane ends with 8 consecutive columns and
// the epilogue stores 16 B per instruction (gemm_big: 2 B); the weight LDS image is swizzled through the DMA
// source addresses (rows XOR 4 in odd k quarters) so those permuted reads stay bank-conflict free.  SiLU keeps the
// natural rows: gate tile 2J and up tile 2J + 1 meet in one lane (8-B stores).
// Reference parity: the projections of xotorch/inference/torch/models/general_mha.py:77-120 / llm_utils.py:513-522.
#include "common.h"
#include "gemm_common.h"
#include "kernels.h"

#include <type_traits>


namespace xot {

// cache-policy bits of the LDS-DMA loads (gfx950 CPol: 1 = sc0, 2 = nt, 16 = sc1), tunable by tools/lab/w4_lab.hip.
// sc1 on both: 3.5-5 % faster than the weights' sc0 + nt streaming hint at 4096 x 4096 x 8192, 4096 x 28672 x 4096
// and 8192^3 (profiles/r5/gemm_w4/lab_cache_bits.log); nt on both is 6-7 % slower
#ifndef W4_XAUX
#define W4_XAUX 16
#endif
#ifndef W4_WAUX
#define W4_WAUX 16
#endif
// k-loop schedule positions (see body below): barrier 1 after MFMA W4_B1 - 1 of half 0, barrier 2 after MFMA
// W4_B2 - 1 of half 1
#ifndef W4_B1
#define W4_B1 32
#endif
#ifndef W4_B2
#define W4_B2 32
#endif
// refill DMA spacing in MFMAs from barrier 1 (0: spread evenly up to barrier 2)
#ifndef W4_DGAP
#define W4_DGAP 0
#endif
#ifndef W4_PROBE
#define W4_PROBE 0
#endif
// fragment reads as inline asm with explicit counted waits (0: compiler-visible loads)
#ifndef W4_ASMRD
#define W4_ASMRD 1
#endif
// fragment reads one per W4_RSP MFMAs
#ifndef W4_RSP
#define W4_RSP 1
#endif
// lab ablations of the k loop (wrong results; timing only, tools/lab/w4_lab.hip): 1 = no refill DMA, 2 = no
// barriers / waits, 4 = no fragment reads, 8 = no loop-end nops (hazard: timing only), 16 = no barrier 1,
// 32 = no vmcnt wait before barrier 2, 64 = no barrier 2
#ifndef W4_ABL
#define W4_ABL 0
#endif

#if W4_PROBE  // lab timing probes (tools/lab/w4_lab.hip): s_memtime at 4 points of every stage, per block and wave
__device__ unsigned long long w4_probe[4096 * 4 * 8 * 4];
#define W4_MARK(P)                                                                                 \
  do {                                                                                             \
    const unsigned long long ts_ = __builtin_amdgcn_s_memtime();                                   \
    w4_probe[((blockIdx.x * 4 + wave) * 8 + (t & 7)) * 4 + (P)] = ts_;                               \
  } while (0)
#else
#define W4_MARK(P) \
  do {             \
  } while (0)
#endif

namespace w4 {
template <int I, int N, class F>
__device__ __forceinline__ void static_for_(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for_<I + 1, N>(f);
  }
}
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) {  // f(integral_constant<int, 0>) .. f(integral_constant<int, N - 1>)
  static_for_<0, N>(f);
}
constexpr int BM = 256, BN = 256, BK = 64;
constexpr int A_EL = BM * BK, STAGE = (BM + BN) * BK;  // bf16 elements per stage buffer (64 KB)
constexpr int SMEM = 2 * STAGE * 2;                     // two stage buffers, 128 KB
}  // namespace w4

// TN (the weight-gradient GEMM dW = dY^T . X on the step's token-major tensors, no dY^T / shuffle(X^T) images in
// HBM): X holds the token operand transposed, Xt [K, M] (k = tokens, ldx apart), W the weight operand likewise,
// Wt [K, N] (ldw apart).  A stage arrives by LDS-DMA as two row-major [64 k][256] images (512-B rows, 16-B granules
// XOR-swizzled by tn_swz(k row) through the source offsets) and every fragment (8 consecutive k of one row or
// column) is two ds_read_b64_tr_b16; the fragment rows are in natural order (no PERM), so the epilogue stores 8 B
// per lane and tile.  The reads are compiler-visible (the explicit read waits below assume one read per fragment).
template <int EPI, bool OUT_F32, bool SPLIT, bool TN = false>
__global__ __launch_bounds__(256, 1) void gemm_w4_kernel(const uint16_t* __restrict__ X, int ldx,
                                                         const uint16_t* __restrict__ W,
                                                         const uint16_t* __restrict__ bias,
                                                         const uint16_t* __restrict__ R, int ldr,
                                                         void* __restrict__ Yv, int ldy, float* __restrict__ ws,
                                                         int M, int N, int K, int S, int group_m, int ldw) {
  using namespace w4;
  static_assert(!TN || (!SPLIT && EPI != EPI_SILU), "TN: weight gradients (plain or residual epilogue)");
  constexpr bool PERM = EPI != EPI_SILU && !TN;
  constexpr bool ASMRD = W4_ASMRD && !TN;
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c = lane & 15;
  const int wm = wave >> 1, wn = wave & 1;

  // ---- tile: bijective XCD remap, split-major, tall grids rastered in groups of group_m row tiles (gemm_big)
  const int mtiles = (M + BM - 1) / BM, ntiles = N / BN;
  const int nwg = mtiles * ntiles * S;
  int b = blockIdx.x;
  {
    const int xcd = b & 7, q = nwg >> 3, r = nwg & 7;
    b = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
  }
  int mt, nt, split;
  {
    const int tiles = mtiles * ntiles;
    split = b / tiles;
    const int bt = b - split * tiles;
    if (group_m > 1 && mtiles >= 2 * group_m) {
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
  const int T_all = K / BK;
  const int t_beg = (int)((long)split * T_all / S), t_end = (int)((long)(split + 1) * T_all / S);
  const int T = t_end - t_beg;

  // ---- LDS-DMA: buffer loads with the whole address in scalar registers but for constant per-lane byte offsets
  // (9 VGPRs): the k stage goes in soffset, the LDS destination in M0 (SALU), so issuing a refill
  // costs the MFMA stream no VALU work.  (Per-issue 64-bit address arithmetic + readfirstlane for M0 -- ~70 VALU
  // per stage -- cost 20 % of the k loop: profiles/r5/gemm_w4/lab_ablation.log.)  Byte offsets are 32-bit: the
  // launcher requires X and this tile's weight rows below 4 GB.
  //   X image: 256 rows x 128 B, 16-B slot (lane % 8) of row r holds logical slot (lane % 8) ^ ((r >> 1) & 7) (gemm_big's
  //   BK = 64 map); instruction d < 8 copies rows 8 (8 wave + d) .. +7, so the swizzle of lane's row is
  //   ((lane >> 4) + 4 (d & 1)) & 7.  Rows past M re-read the last; their outputs are masked.
  //   W image: (16-row group, k32 block) 1-KB blocks in order (group * 2 + block); instruction 8 + i copies block
  //   i & 1 of group 4 wave + i / 2.  PERM: lane l of a block loads granule (kq = l >> 4, row (l & 15) ^ 4 (kq & 1)).
  auto aswz = [](int row) -> int { return (row >> 1) & 7; };
  const int swave = __builtin_amdgcn_readfirstlane(wave);
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc((void*)X, (short)0, -1, 0x00020000);
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(W + (size_t)((n0 >> 4) + 4 * swave) * (K / 128) * 2048), (short)0, -1, 0x00020000);
  int xvo[8], wvo;  // per-lane byte offsets: X per instruction (row clamp), W one for all (the rest is scalar)
  int tvo[8];       // TN: the W operand's per-instruction offsets
  // TN: instruction q = 8 wave + d of either operand copies k rows 2q, 2q + 1 of the stage (512 B each): lane l ->
  // k row 2q + l / 32, physical granule l % 32 holding logical granule (l % 32) ^ tn_swz(k row).  tn_swz puts the
  // 8 rows a 32-lane half reads transposed (rows 8 g + 0..3 of two lane groups) on 8 distinct 8-bank octets.
  auto tn_swz = [](int krow) -> int { return 2 * ((krow & 3) | (((krow >> 3) & 1) << 2)); };
  if constexpr (TN) {
#pragma unroll
    for (int d = 0; d < 8; ++d) {
      const int kr = 2 * (8 * wave + d) + (lane >> 5), lg = (lane & 31) ^ tn_swz(kr);
      xvo[d] = (int)(((unsigned)kr * (unsigned)ldx + (unsigned)(m0 + 8 * lg)) * 2u);
      tvo[d] = (int)(((unsigned)kr * (unsigned)ldw + (unsigned)(n0 + 8 * lg)) * 2u);
    }
    wvo = 0;
  } else {
    const int xr0 = 64 * wave + (lane >> 3);
    const int xslot[2] = {((lane & 7) ^ ((lane >> 4) & 7)) * 8, ((lane & 7) ^ (((lane >> 4) + 4) & 7)) * 8};
#pragma unroll
    for (int d = 0; d < 8; ++d)
      xvo[d] = (int)(((unsigned)min(m0 + xr0 + 8 * d, M - 1) * (unsigned)ldx + xslot[d & 1]) * 2u);
    wvo = (PERM ? (((lane >> 4) * 16 + ((lane & 15) ^ (4 * ((lane >> 4) & 1)))) * 8) : lane * 8) * 2;
#pragma unroll
    for (int d = 0; d < 8; ++d) tvo[d] = 0;
  }
  const __amdgpu_buffer_rsrc_t trs = __builtin_amdgcn_make_buffer_rsrc((void*)W, (short)0, -1, 0x00020000);
  auto issue = [&](int t, int buf, int d) {  // LDS-DMA instruction d (0..15) of this wave for k stage t
    typedef __attribute__((address_space(3))) void* lds_t;
    uint16_t* As = smem + buf * STAGE;
    if constexpr (TN) {
      if (d < 8)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (lds_t)(As + (8 * swave + d) * 512), 16, xvo[d], t * (BK * 2) * ldx,
                                                 0, W4_XAUX);
      else
        __builtin_amdgcn_raw_ptr_buffer_load_lds(trs, (lds_t)(As + A_EL + (8 * swave + d - 8) * 512), 16, tvo[d - 8],
                                                 t * (BK * 2) * ldw, 0, W4_WAUX);
      return;
    }
    if (d < 8) {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (lds_t)(As + (8 * swave + d) * 512), 16, xvo[d], t * (BK * 2), 0,
                                               W4_XAUX);
    } else {
      const int i = d - 8;  // group 4 wave + i / 2, block i & 1
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs, (lds_t)(As + A_EL + (8 * swave + i) * 512), 16, wvo,
                                               t * 2048 + (i >> 1) * (K / 128) * 4096 + (i & 1) * 1024, 0, W4_WAUX);
    }
  };

  // ---- fragment offsets (elements inside a stage buffer).  Token tile i: base + 1024 i (16 rows of 64); its swizzle
  // ((16 i + c) >> 1) & 7 = (c >> 1) & 7 does not depend on i.  Weight tile j: pair base (j & 1) + 2048 (j >> 1).
  int xo[2], wo[2][2];
  {
    const int row = wm * 128 + c;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) xo[s2] = row * BK + (((4 * s2 + g) ^ aswz(row)) * 8);
  }
#pragma unroll
  for (int jj = 0; jj < 2; ++jj) {
    int grp, pos;
    if constexpr (PERM) {
      const int rho = 8 * (c >> 2) + (c & 3) + 4 * jj;  // row of the 32-row block of tiles (2J, 2J + 1)
      grp = wn * 8 + (rho >> 4);
      pos = g * 16 + ((rho & 15) ^ (4 * (g & 1)));
    } else {
      grp = wn * 8 + jj;
      pos = g * 16 + c;
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) wo[jj][s2] = A_EL + (grp * 2 + s2) * 512 + pos * 8;
  }

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  s16x8 wf[2][8], xf[2][8];

  // The k loop's waits as the s_waitcnt builtin, not inline asm: the compiler's wait-count model then sees them.
  // With an opaque asm lgkmcnt(0) it still counted half 1's 16 reads as in flight at the loop top, more than the
  // 4-bit counter can name beside the 16 read-ahead reads, and fell back to lgkmcnt(0) before the first MFMA of
  // every stage (waiting for the whole read-ahead) instead of the lgkmcnt(14) its two operands need.
  // gfx950 encoding: vmcnt[3:0] | expcnt[6:4] | lgkmcnt[11:8] | vmcnt[5:4] << 14.
  auto lgkm0 = []() {  // lgkmcnt(0)
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_waitcnt(0xC07F);
    asm volatile("" ::: "memory");
  };
  auto vm16 = []() {  // vmcnt(16): this wave's older stage landed, the 16 refill DMAs stay in flight
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_waitcnt((16 & 15) | (7 << 4) | (15 << 8) | ((16 >> 4) << 14));
    asm volatile("" ::: "memory");
  };
  auto bar = []() {  // raw barrier: LDS-DMA stays in flight; the asm statements fence the compiler
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  // MFMA u (0..63) of k half h: weight tile j = u / 8 against token tile i = u % 8.  Inline asm with the accumulator
  // tied to its AGPR quad: with the builtin the compiler kept moving the 256 accumulators between AGPRs and VGPRs
  // inside the k loop (~500 v_accvgpr moves per stage).  The asm is invisible to the hazard recognizer: the
  // epilogue waits for the last MFMAs explicitly.
  auto mma = [&](int h, int u) {
    const int j = u >> 3, i = u & 7;
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[i][j]) : "v"(wf[h][j]), "v"(xf[h][i]));
  };
  // Keep the 16 fragments of k half h alive up to this point.  The MFMAs are inline asm, so the hazard recognizer
  // does not know they read their A / B registers over several cycles: a VALU write to a fragment register right
  // after the MFMA that last read it (the compiler reused dead fragment registers for address arithmetic one MFMA
  // later) corrupted the product.  Fragment registers stay allocated for a whole phase, and the loop end pads the
  // one boundary where a VALU may follow the last reader directly.
  auto keep = [&](int h) {
    asm volatile("" ::"v"(wf[h][0]), "v"(wf[h][1]), "v"(wf[h][2]), "v"(wf[h][3]), "v"(wf[h][4]), "v"(wf[h][5]),
                 "v"(wf[h][6]), "v"(wf[h][7]), "v"(xf[h][0]), "v"(xf[h][1]), "v"(xf[h][2]), "v"(xf[h][3]),
                 "v"(xf[h][4]), "v"(xf[h][5]), "v"(xf[h][6]), "v"(xf[h][7]));
  };
  // fragment read f (0..15) of k half h, in the order the MFMAs consume them (weight tile 0, token tiles 0..7,
  // weight tiles 1..7): the first MFMA of a half waits for 2 reads (counted lgkmcnt), not for all 16
#if W4_ASMRD
  // Fragment reads as inline asm with explicit counted waits (before MFMAs 0..8 and 16 of a stage): the
  // compiler's wait-count model, merging the prologue's and the previous stage's read-ahead at the loop header,
  // put lgkmcnt(0) before every stage's first MFMA -- the whole 16-read read-ahead exposed each stage.  Byte
  // addresses: one base per (operand, k half) plus the stage buffer's 64 KB, tile offsets as immediates.
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint16_t*)smem;
  auto rd_asm = [&](int buf, int h, int f) {
    const uint32_t bo = lds0 + (uint32_t)buf * (STAGE * 2);
    if (f == 0 || f > 8) {
      const int j = f == 0 ? 0 : f - 8;
      const uint32_t a = bo + (uint32_t)wo[j & 1][h] * 2;
      switch (j >> 1) {  // immediate offset 4096 (j / 2) bytes
        case 0: asm volatile("ds_read_b128 %0, %1" : "=v"(wf[h][j]) : "v"(a)); break;
        case 1: asm volatile("ds_read_b128 %0, %1 offset:4096" : "=v"(wf[h][j]) : "v"(a)); break;
        case 2: asm volatile("ds_read_b128 %0, %1 offset:8192" : "=v"(wf[h][j]) : "v"(a)); break;
        default: asm volatile("ds_read_b128 %0, %1 offset:12288" : "=v"(wf[h][j]) : "v"(a)); break;
      }
    } else {
      const int i = f - 1;
      const uint32_t a = bo + (uint32_t)xo[h] * 2;
      switch (i) {  // immediate offset 2048 i bytes
        case 0: asm volatile("ds_read_b128 %0, %1" : "=v"(xf[h][i]) : "v"(a)); break;
        case 1: asm volatile("ds_read_b128 %0, %1 offset:2048" : "=v"(xf[h][i]) : "v"(a)); break;
        case 2: asm volatile("ds_read_b128 %0, %1 offset:4096" : "=v"(xf[h][i]) : "v"(a)); break;
        case 3: asm volatile("ds_read_b128 %0, %1 offset:6144" : "=v"(xf[h][i]) : "v"(a)); break;
        case 4: asm volatile("ds_read_b128 %0, %1 offset:8192" : "=v"(xf[h][i]) : "v"(a)); break;
        case 5: asm volatile("ds_read_b128 %0, %1 offset:10240" : "=v"(xf[h][i]) : "v"(a)); break;
        case 6: asm volatile("ds_read_b128 %0, %1 offset:12288" : "=v"(xf[h][i]) : "v"(a)); break;
        default: asm volatile("ds_read_b128 %0, %1 offset:14336" : "=v"(xf[h][i]) : "v"(a)); break;
      }
    }
  };
#endif
  auto rd_c = [&](int buf, int h, int f) {
    const uint16_t* Ls = smem + buf * STAGE;
    const int j = f == 0 ? 0 : (f <= 8 ? -1 : f - 8);
    if (j >= 0) wf[h][j] = ld16(Ls + wo[j & 1][h] + 2048 * (j >> 1));
    else xf[h][f - 1] = ld16(Ls + xo[h] + 1024 * (f - 1));
  };
  // TN fragments: element offsets (k half 0, rows 8 g + (c >> 2)) of token tile i and weight tile j in their images;
  // k half h is 32 rows further, the second read 4 rows (tn_swz ignores bit 2 of the row: same swizzle).  Lane
  // 4 q + p of a 16-lane group addresses k row q of the block, columns 4 p .. 4 p + 3; lane c receives column c.
  int ta[8], tb[8];
  if constexpr (TN) {
    const int kr = 8 * g + (c >> 2), sw = tn_swz(kr);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int xc = wm * 128 + 16 * i + 4 * (c & 3), wc = wn * 128 + 16 * i + 4 * (c & 3);
      ta[i] = kr * 256 + ((((xc >> 3) ^ sw) << 3) | (xc & 7));
      tb[i] = A_EL + kr * 256 + ((((wc >> 3) ^ sw) << 3) | (wc & 7));
    }
  }
  // As inline asm: compiler-visible LDS reads after LDS-DMA issues made hipcc drain vmcnt(0) -- the whole refill in
  // flight -- before the first read of every stage.  Waits: the k loop's s_waitcnt lgkmcnt(15) before MFMAs 0 .. 16.
  const uint32_t tlds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint16_t*)smem;
  auto rd_tn = [&](int buf, int h, int f) {
    const int j = f == 0 ? 0 : (f <= 8 ? -1 : f - 8);
    const uint32_t a = tlds0 + (uint32_t)buf * (STAGE * 2) + (uint32_t)(j >= 0 ? tb[j] : ta[f - 1]) * 2;
    s16x4 lo, hi;
    if (h == 0) {
      asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo) : "v"(a));
      asm volatile("ds_read_b64_tr_b16 %0, %1 offset:2048" : "=v"(hi) : "v"(a));
    } else {
      asm volatile("ds_read_b64_tr_b16 %0, %1 offset:16384" : "=v"(lo) : "v"(a));
      asm volatile("ds_read_b64_tr_b16 %0, %1 offset:18432" : "=v"(hi) : "v"(a));
    }
    const s16x8 v = s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    if (j >= 0) wf[h][j] = v;
    else xf[h][f - 1] = v;
  };
  auto rd = [&](int buf, int h, int f) {
    if constexpr (TN) {
      rd_tn(buf, h, f);
    } else {
#if W4_ASMRD
      rd_asm(buf, h, f);
#else
      rd_c(buf, h, f);
#endif
    }
  };

  {  // T >= 1 (S <= K / 64).  Prologue without branches: stage 1 (stage 0 again when T == 1) into buffer 1
#pragma unroll
    for (int d = 0; d < 16; ++d) issue(t_beg, 0, d);
#pragma unroll
    for (int d = 0; d < 16; ++d) issue(t_beg + min(1, T - 1), 1, d);
    wait_vm<16>();
    bar();
#pragma unroll
    for (int f = 0; f < 16; ++f) {  // in consumption order, as in the loop
      rd(0, 0, f);
      __builtin_amdgcn_sched_barrier(0);
    }

    // one 64-deep stage.  Every stage refills and reads ahead unconditionally -- past the end stage T - 1 again,
    // into a buffer no later stage reads -- so the k loop is straight-line code: a branch inside it made the
    // register allocator shuffle the 256 accumulators between AGPR quads at the join.
    // Global MFMA index v = 0..127 of a stage (half v / 64, MFMA v % 64).  Half 1's 16 fragment reads go under the
    // first 16; after MFMA B1 - 1 every wave has them (lgkmcnt(0) + barrier) and this buffer is free; the 16 refill
    // DMAs of stage t + 2 spread evenly over MFMAs B1 .. 64 + B2 - 1; after MFMA 64 + B2 - 1 stage t + 1 has landed
    // for this wave (vmcnt(16): the refill stays in flight) and for every wave (barrier), and its half-0 fragments
    // are read under the next 16 MFMAs, in the order the next stage consumes them.
    constexpr int B1 = W4_B1, B2 = W4_B2, SPAN = 64 - B1 + B2, DGAP = W4_DGAP, RSP = W4_RSP;
    static_assert(16 * RSP <= B1 && B2 + 16 * RSP <= 64, "fragment reads between the barriers");
    static_assert(DGAP == 0 || B1 + DGAP * 15 < 64 + B2, "refill DMAs before barrier 2");
    static_assert(B1 >= 17 && B1 <= 64 && B2 >= 8 && B2 <= 48, "schedule positions");
    static_assert(!W4_ASMRD || RSP == 1, "the explicit read waits assume one read per MFMA");
    auto body = [&](int t) {
      const int buf = t & 1;
      const int tr = t_beg + min(t + 2, T - 1);
      W4_MARK(0);
      static_for<128>([&](auto vc) {  // compile-time v: every condition below folds away
        constexpr int v = decltype(vc)::value;
        constexpr int h = v >> 6, u = v & 63;
#if W4_ASMRD
        if constexpr (ASMRD) {
        // the read-ahead (16 reads, consumption order) and the v half-1 reads issued since: MFMA v <= 8 needs
        // read-ahead v + 1 (w0 + x_v, then w1) -> at most 14 younger reads in flight; from MFMA 16 on (w2..w7)
        // the whole read-ahead -> 15 (stricter than needed, the counter's maximum)
        if constexpr (v <= 8) asm volatile("s_waitcnt lgkmcnt(14)" ::: "memory");
        if constexpr (v == 16) asm volatile("s_waitcnt lgkmcnt(15)" ::: "memory");
        }
#endif
        // TN: 32 read-ahead reads (two per fragment, consumption order) then two half-1 reads per MFMA from MFMA 0:
        // before MFMA v <= 16 at most 15 reads in flight means reads 0 .. 16 + 2v are done (LDS reads retire in
        // order), which covers fragment v + 1 (x_v, reads 2v + 2, 2v + 3) up to v = 7, w1 (reads 18, 19) at 8 .. 15
        // and, at 16, all 32 read-ahead reads
        if constexpr (TN && v <= 16) asm volatile("s_waitcnt lgkmcnt(15)" ::: "memory");
        mma(h, u);
        if constexpr (!(W4_ABL & 4) && v % RSP == 0 && v < 16 * RSP) rd(buf, 1, v / RSP);
        if constexpr (!(W4_ABL & 4) && v >= 64 + B2 && (v - 64 - B2) % RSP == 0 && v < 64 + B2 + 16 * RSP)
          rd(buf ^ 1, 0, (v - 64 - B2) / RSP);
        if constexpr (!(W4_ABL & 1) && v >= B1 && v < 64 + B2) {
          static_for<16>([&](auto kc) {  // refill DMA k after MFMA B1 + ((k + 1) SPAN) / 16 - 1
            constexpr int k = decltype(kc)::value;
            if constexpr ((DGAP ? B1 + DGAP * k : B1 + ((k + 1) * SPAN) / 16 - 1) == v) issue(tr, buf, k);
          });
        }
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (!(W4_ABL & 2) && v == B1 - 1) {
          lgkm0();
          if constexpr (!(W4_ABL & 16)) bar();
          W4_MARK(1);
        }
        if constexpr (!(W4_ABL & 2) && v == 64 + B2 - 1) {
          if constexpr (!(W4_ABL & 32)) vm16();
          if constexpr (!(W4_ABL & 64)) bar();
          W4_MARK(2);
        }
        if constexpr (v == 63) keep(0);
      });
      keep(1);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (!(W4_ABL & 8))
        asm volatile("s_nop 7\n s_nop 7" ::: "memory");  // VALU after the last reader of a half-1 register (loop top)
      __builtin_amdgcn_sched_barrier(0);
      W4_MARK(3);
    };
    // One loop body for every stage, the last included (its read-ahead reads a re-loaded stage nobody uses): a
    // peeled last body got its own accumulator allocation, and the AGPR shuffle the allocator put between the loop
    // and it raced the inline-asm MFMAs it cannot see.
    for (int t = 0; t < T; ++t) body(t);
    wait_vm<0>();  // the last refills (re-loads of stage T - 1 nobody reads) land before the wave ends
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // ... and the last read-ahead, before registers are reused
  }

  // the last MFMAs (inline asm: the hazard recognizer does not see them) retire before the epilogue reads their
  // accumulators; the scheduling barrier keeps those reads (no dependence on the nops) from moving above them
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);

  // ---- epilogue.  Lane (g, c): token row trow(i) = m0 + 128 wm + 16 i + c; PERM: columns 32 J + 8 g .. +8 of the
  // wave's 128 from tiles (2J, 2J + 1); SiLU: output columns 16 J + 4 g .. +4 (gate tile 2J, up tile 2J + 1).
  const int rbase = m0 + wm * 128 + c;
  const int cbase = n0 + wn * 128;
  if constexpr (SPLIT) {  // raw fp32 partial slabs, in the natural or permuted column order of the lane
    float* slab = ws + (size_t)split * M * N;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = rbase + 16 * i;
      if (m >= M) continue;
      float* row = slab + (size_t)m * N + cbase;
#pragma unroll
      for (int J = 0; J < 4; ++J) {
        if constexpr (PERM) {
          *reinterpret_cast<f32x4*>(row + 32 * J + 8 * g) = acc[i][2 * J];
          *reinterpret_cast<f32x4*>(row + 32 * J + 8 * g + 4) = acc[i][2 * J + 1];
        } else {
          *reinterpret_cast<f32x4*>(row + 32 * J + 4 * g) = acc[i][2 * J];
          *reinterpret_cast<f32x4*>(row + 32 * J + 16 + 4 * g) = acc[i][2 * J + 1];
        }
      }
    }
  } else if constexpr (TN) {  // natural column order: lane (g, c) holds columns cbase + 16 j + 4 g .. +4 of token row
    typedef short s16x4_t __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = rbase + 16 * i;
      if (m >= M) continue;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int col = cbase + 16 * j + 4 * g;
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = acc[i][j][r];
        if constexpr (EPI == EPI_RESID) {
          const s16x4_t rv = *reinterpret_cast<const s16x4_t*>(R + (size_t)m * ldr + col);
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] += bf2f(rv[r]);
        }
        if constexpr (OUT_F32) {
          *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(Yv) + (size_t)m * ldy + col) = f32x4{v[0], v[1], v[2], v[3]};
        } else {
          s16x4_t o;
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = (short)f2bf(v[r]);
          *reinterpret_cast<s16x4_t*>(reinterpret_cast<uint16_t*>(Yv) + (size_t)m * ldy + col) = o;
        }
      }
    }
  } else if constexpr (PERM) {
    s16x8 bv[4];
    if (bias != nullptr) {
#pragma unroll
      for (int J = 0; J < 4; ++J) bv[J] = ld16(bias + cbase + 32 * J + 8 * g);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = rbase + 16 * i;
      s16x8 rv[4];
      if constexpr (EPI == EPI_RESID) {
        const int mr = min(m, M - 1);
#pragma unroll
        for (int J = 0; J < 4; ++J) rv[J] = ld16(R + (size_t)mr * ldr + cbase + 32 * J + 8 * g);
      }
      if (m < M) {
#pragma unroll
        for (int J = 0; J < 4; ++J) {
          float v[8];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            v[r] = acc[i][2 * J][r];
            v[4 + r] = acc[i][2 * J + 1][r];
          }
          const int col = cbase + 32 * J + 8 * g;
          {
            if (bias != nullptr) {
#pragma unroll
              for (int e = 0; e < 8; ++e) v[e] += bf2f(bv[J][e]);
            }
            if constexpr (EPI == EPI_RESID) {
#pragma unroll
              for (int e = 0; e < 8; ++e) v[e] += bf2f(rv[J][e]);
            }
            if constexpr (OUT_F32) {
              float* p = reinterpret_cast<float*>(Yv) + (size_t)m * ldy + col;
              *reinterpret_cast<f32x4*>(p) = f32x4{v[0], v[1], v[2], v[3]};
              *reinterpret_cast<f32x4*>(p + 4) = f32x4{v[4], v[5], v[6], v[7]};
            } else {
              s16x8 o;
#pragma unroll
              for (int e = 0; e < 8; ++e) o[e] = (short)f2bf(v[e]);
              st16(reinterpret_cast<uint16_t*>(Yv) + (size_t)m * ldy + col, o);
            }
          }
        }
      }
    }
  } else {  // SiLU: natural rows, gate tile 2J / up tile 2J + 1 -> 4 output columns per lane
    const int obase = cbase / 2;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = rbase + 16 * i;
      if (m >= M) continue;
#pragma unroll
      for (int J = 0; J < 4; ++J) {
        const int gcol = cbase + 32 * J + 4 * g;  // gate rows of this lane (16-row interleaved gate / up groups)
        float o4[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float gv = acc[i][2 * J][r], uv = acc[i][2 * J + 1][r];
          if (bias != nullptr) {
            gv += bf2f(bias[gcol + r]);
            uv += bf2f(bias[gcol + 16 + r]);
          }
          o4[r] = silu(gv) * uv;
        }
        const int col = obase + 16 * J + 4 * g;
        if constexpr (OUT_F32) {
          *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(Yv) + (size_t)m * ldy + col) =
              f32x4{o4[0], o4[1], o4[2], o4[3]};
        } else {
          typedef short s16x4_t __attribute__((ext_vector_type(4)));
          s16x4_t o;
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = (short)f2bf(o4[r]);
          *reinterpret_cast<s16x4_t*>(reinterpret_cast<uint16_t*>(Yv) + (size_t)m * ldy + col) = o;
        }
      }
    }
  }
}

template <int EPI, bool F32, bool SPLIT>
static void w4_launch(const uint16_t* X, int ldx, const uint16_t* W, const uint16_t* bias, const uint16_t* R, int ldr,
                      void* Y, int ldy, float* ws, int M, int N, int K, int S, int group_m, hipStream_t st) {
  auto kern = gemm_w4_kernel<EPI, F32, SPLIT>;
  static bool attr =
      hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, w4::SMEM) == hipSuccess;
  (void)attr;
  const int nwg = ((M + 255) / 256) * (N / 256) * S;
  kern<<<nwg, 256, w4::SMEM, st>>>(X, ldx, W, bias, R, ldr, Y, ldy, ws, M, N, K, S, group_m, 0);
}

template <int EPI, bool F32>
static void w4_tn_launch(const uint16_t* Xt, int ldx, const uint16_t* Wt, int ldw, const uint16_t* R, int ldr, void* Y,
                         int ldy, int M, int N, int K, int group_m, hipStream_t st) {
  auto kern = gemm_w4_kernel<EPI, F32, false, true>;
  static bool attr =
      hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, w4::SMEM) == hipSuccess;
  (void)attr;
  kern<<<(M / 256) * (N / 256), 256, w4::SMEM, st>>>(Xt, ldx, Wt, nullptr, R, ldr, Y, ldy, nullptr, M, N, K, 1,
                                                       group_m, ldw);
}

// Weight gradients on the token-major operands: Y [M, N] (+)= Xt^T . Wt, Xt [K, M] (ldx), Wt [K, N] (ldw); M, N
// multiples of 256, K of 64; plain (bf16 / fp32) or residual (bf16, in place when R == Y) epilogue.
int launch_gemm_w4_tn(const uint16_t* Xt, int ldx, const uint16_t* Wt, int ldw, const uint16_t* R, int ldr, void* Y,
                      int ldy, bool out_f32, int epi, int M, int N, int K, int group_m, hipStream_t st) {
  if (M <= 0 || N <= 0) return 0;
  if (M % 256 || N % 256 || K % 64 || K <= 0 || ldx % 8 || ldw % 8) return -1;
  if ((size_t)K * ldx * 2 >= (1ull << 31) || (size_t)K * ldw * 2 >= (1ull << 31)) return -1;  // 32-bit offsets
  if (epi == EPI_RESID) {
    if (out_f32) return -1;
    w4_tn_launch<EPI_RESID, false>(Xt, ldx, Wt, ldw, R, ldr, Y, ldy, M, N, K, group_m, st);
  } else if (epi == EPI_NONE) {
    if (out_f32) w4_tn_launch<EPI_NONE, true>(Xt, ldx, Wt, ldw, R, ldr, Y, ldy, M, N, K, group_m, st);
    else w4_tn_launch<EPI_NONE, false>(Xt, ldx, Wt, ldw, R, ldr, Y, ldy, M, N, K, group_m, st);
  } else {
    return -1;
  }
  return 0;
}

// Tile code 4256 of launch_gemm_big.  S > 1 writes fp32 slabs (reduced by the caller's reduce kernel).
int launch_gemm_w4(const uint16_t* X, int ldx, const uint16_t* W, const uint16_t* bias, const uint16_t* R, int ldr,
                   void* Y, int ldy, bool out_f32, int epi, float* ws, int M, int N, int K, int S, int group_m,
                   hipStream_t st) {
  if (M <= 0) return 0;
  if (N % 256 != 0 || K % 128 != 0 || S < 1 || S > K / 64) return -1;
  if ((size_t)M * ldx * 2 >= (1ull << 32)) return -1;  // 32-bit byte offsets of the LDS-DMA buffer loads
  if (S > 1) {
    if (ws == nullptr) return -1;
    if (epi == EPI_SILU) w4_launch<EPI_SILU, true, true>(X, ldx, W, bias, R, ldr, Y, ldy, ws, M, N, K, S, group_m, st);
    else w4_launch<EPI_NONE, true, true>(X, ldx, W, bias, R, ldr, Y, ldy, ws, M, N, K, S, group_m, st);
    return 0;
  }
  if (epi == EPI_SILU) {
    if (out_f32) w4_launch<EPI_SILU, true, false>(X, ldx, W, bias, R, ldr, Y, ldy, ws, M, N, K, 1, group_m, st);
    else w4_launch<EPI_SILU, false, false>(X, ldx, W, bias, R, ldr, Y, ldy, ws, M, N, K, 1, group_m, st);
  } else if (epi == EPI_RESID) {
    if (out_f32) return -1;
    w4_launch<EPI_RESID, false, false>(X, ldx, W, bias, R, ldr, Y, ldy, ws, M, N, K, 1, group_m, st);
  } else {
    if (out_f32) w4_launch<EPI_NONE, true, false>(X, ldx, W, bias, R, ldr, Y, ldy, ws, M, N, K, 1, group_m, st);
    else w4_launch<EPI_NONE, false, false>(X, ldx, W, bias, R, ldr, Y, ldy, ws, M, N, K, 1, group_m, st);
  }
  return 0;
}

}  // namespace xot

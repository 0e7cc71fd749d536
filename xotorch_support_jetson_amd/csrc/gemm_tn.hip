// Weight-gradient GEMM straight from the activations' token-major layout:  C[M,N] (+)= A[K,M]^T . B[K,N]
//
// In the training step dW = dY^T . X with dY [T, N_out] and X [T, K_in] both token-major, the reduction (the
// tokens) being each operand's SLOW index.  The other large GEMMs take the reduction index fastest, so the
// round-3 step first relaid both operands per micro-batch (dY^T and shuffle(X^T): ~3.5 % of the 8B step in two
// transpose kernels plus their HBM round trips).  This kernel reads them as they are:
//   * tile 256 (m) x 256 (n) x 64 (tokens), 8 waves as 2 x 4, wave tile 128 x 64 = 8 x 4 MFMA 16x16x32 tiles
//   * both operands staged by LDS-DMA (global_load_lds_dwordx4) as [64 tokens][256 columns] images with
//     512-B rows, two stages (128 KB); per stage 4 + 4 1-KB instructions per wave
//   * MFMA operands come out of the images with ds_read_b64_tr_b16 (cdna_hip_programming.md T10): a 16-lane
//     group reads 4 token rows x 16 columns and lane i receives column i's 4 tokens -- two such reads give the
//     8 consecutive tokens of the 16x16x32 A / B fragment of lane (g, c) (column c, tokens 8g .. 8g + 7)
//   * 16-B chunk of row r stored at chunk ^ 2h(r), h(r) = (r & 3) | ((r >> 3) & 1) << 2: the 8 token rows a
//     32-lane half reads together (r0 .. r0+3 and r0+8 .. r0+11) land in 8 distinct 32-B bank groups; the
//     swizzle is applied to the per-lane global source address, so the DMA image stays lane-linear
//   * XCD-aware, M-grouped tile order as gemm_big; epilogue: plain store or residual add (the bf16 gradient
//     accumulator of the micro-batches), in place
// Reference op: the weight gradients of the projections a trainer of xotorch/inference/torch/models/
// general_mha.py:77-120 / llm_utils.py:513-522 would run through autograd (the reference never trained).
#include "common.h"
#include "gemm_common.h"
#include "kernels.h"

namespace xot {

namespace {
typedef __attribute__((address_space(3))) s16x4* lds_s16x4_tn;

__device__ __forceinline__ s16x4 tr_read4(const uint16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_tn)(p));
}

constexpr int TN_BM = 256, TN_BN = 256, TN_BK = 64, TN_WM = 2, TN_WN = 4;
constexpr int TN_MT = TN_BM / (16 * TN_WM), TN_NT = TN_BN / (16 * TN_WN);  // 8 x 4 MFMA tiles per wave
constexpr int TN_ROW = 256;                 // elements per image row (= BM = BN)
constexpr int TN_IMG = TN_BK * TN_ROW;      // elements per operand image
constexpr int TN_STAGE = 2 * TN_IMG;        // A image then B image
constexpr int TN_INSTR = TN_IMG * 2 / 1024 / 8;  // 1-KB DMA instructions per wave per operand per stage (4)

__device__ __forceinline__ int tn_swz(int row) { return (((row & 3) | (((row >> 3) & 1) << 2)) << 1); }
}  // namespace

template <int EPI, bool OUT_F32>
__global__ __launch_bounds__(512, 1) void gemm_tn_kernel(const uint16_t* __restrict__ A, int lda,
                                                         const uint16_t* __restrict__ B, int ldb,
                                                         const uint16_t* __restrict__ R, int ldr,
                                                         void* __restrict__ Cv, int ldc, int M, int N, int K) {
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c = lane & 15;
  const int wm = wave / TN_WN, wn = wave % TN_WN;

  // ---- tile: bijective XCD remap, then groups of 4 row tiles x every column tile, column-major in a group
  const int mtiles = M / TN_BM, ntiles = N / TN_BN, nwg = mtiles * ntiles;
  int b = blockIdx.x;
  {
    const int xcd = b & 7, q = nwg >> 3, r = nwg & 7;
    b = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
  }
  constexpr int GROUP_M = 4;
  int mt, nt;
  if (mtiles >= 2 * GROUP_M) {
    const int per = GROUP_M * ntiles, grp = b / per, first = grp * GROUP_M;
    const int gm = min(mtiles - first, GROUP_M), rr = b - grp * per;
    mt = first + rr % gm;
    nt = rr / gm;
  } else {
    mt = b % mtiles;
    nt = b / mtiles;
  }
  const int m0 = mt * TN_BM, n0 = nt * TN_BN;

  // ---- LDS-DMA sources: instruction i of wave w fills image rows 2 (4w + i) and +1; lane -> row + lane / 32,
  // physical chunk lane % 32 holding logical chunk (lane % 32) ^ swz(row)
  const uint16_t* asrc[TN_INSTR];
  const uint16_t* bsrc[TN_INSTR];
#pragma unroll
  for (int i = 0; i < TN_INSTR; ++i) {
    const int row = 2 * (TN_INSTR * wave + i) + (lane >> 5);
    const int chunk = (lane & 31) ^ tn_swz(row);
    asrc[i] = A + (size_t)row * lda + m0 + chunk * 8;
    bsrc[i] = B + (size_t)row * ldb + n0 + chunk * 8;
  }
  auto issue = [&](int t, int buf) {
    uint16_t* As = smem + buf * TN_STAGE;
    uint16_t* Bs = As + TN_IMG;
    const size_t ka = (size_t)t * TN_BK * lda, kb = (size_t)t * TN_BK * ldb;
#pragma unroll
    for (int i = 0; i < TN_INSTR; ++i) glds16<0>(asrc[i] + ka, As + (TN_INSTR * wave + i) * 512);
#pragma unroll
    for (int i = 0; i < TN_INSTR; ++i) glds16<0>(bsrc[i] + kb, Bs + (TN_INSTR * wave + i) * 512);
  };

  // ---- transposed fragment reads.  Lane 4q + p of a 16-lane group addresses row r0 + q, columns col0 + 4p ..
  // +3 (chunk col0 / 8 + p / 2, byte 8 (p & 1)); the group's lane i gets column col0 + i of those 4 rows.
  const int q4 = c >> 2, p4 = c & 3;
  auto tr_off = [&](int r0, int col0) -> int {
    const int row = r0 + q4;
    return row * TN_ROW + ((((col0 >> 3) + (p4 >> 1)) ^ tn_swz(row)) << 3) + 4 * (p4 & 1);
  };
  // fragment of column tile col0 (16 columns), k-step s: tokens 32 s + 8 g .. + 8 -> s16x8
  auto frag = [&](const uint16_t* img, int col0, int s) -> s16x8 {
    const int r0 = 32 * s + 8 * g;
    const s16x4 lo = tr_read4(img + tr_off(r0, col0)), hi = tr_read4(img + tr_off(r0 + 4, col0));
    return s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  };

  f32x4 acc[TN_MT][TN_NT];
#pragma unroll
  for (int i = 0; i < TN_MT; ++i)
#pragma unroll
    for (int j = 0; j < TN_NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int mw = wm * (TN_MT * 16), nw = wn * (TN_NT * 16);
  constexpr int LDPF = 3;
  auto compute = [&](int buf) {
    const uint16_t* As = smem + buf * TN_STAGE;
    const uint16_t* Bs = As + TN_IMG;
#pragma unroll
    for (int s = 0; s < TN_BK / 32; ++s) {
      s16x8 bf[TN_NT];
#pragma unroll
      for (int j = 0; j < TN_NT; ++j) bf[j] = frag(Bs, nw + 16 * j, s);
      s16x8 af[LDPF];
#pragma unroll
      for (int u = 0; u < LDPF; ++u) af[u] = frag(As, mw + 16 * u, s);
#pragma unroll
      for (int i = 0; i < TN_MT; ++i) {
        const s16x8 cur = af[i % LDPF];
        if (i + LDPF < TN_MT) af[i % LDPF] = frag(As, mw + 16 * (i + LDPF), s);
#pragma unroll
        for (int j = 0; j < TN_NT; ++j) acc[i][j] = mfma16(cur, bf[j], acc[i][j]);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };
  auto barrier = []() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  const int T = K / TN_BK;
  issue(0, 0);
  wait_vm<0>();
  barrier();
  for (int t = 0; t < T; ++t) {
    if (t + 1 < T) issue(t + 1, (t + 1) & 1);  // the other buffer: every wave passed last iteration's barrier
    compute(t & 1);
    wait_vm<0>();
    barrier();
  }

  // ---- epilogue: rows m0 + mw + 16 i + 4 g + r, columns n0 + nw + 16 j + c
  const int rbase = m0 + mw, cbase = n0 + nw;
#pragma unroll
  for (int j = 0; j < TN_NT; ++j) {
    const int col = cbase + 16 * j + c;
#pragma unroll
    for (int i0 = 0; i0 < TN_MT; i0 += TN_MT / 2) {
      float rv[TN_MT / 2][4];
      if constexpr (EPI == EPI_RESID) {  // residuals of the row group loaded up front (one latency)
#pragma unroll
        for (int i = 0; i < TN_MT / 2; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) rv[i][r] = bf2f(R[(size_t)(rbase + 16 * (i0 + i) + 4 * g + r) * ldr + col]);
      }
#pragma unroll
      for (int i = 0; i < TN_MT / 2; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = rbase + 16 * (i0 + i) + 4 * g + r;
          float v = acc[i0 + i][j][r];
          if constexpr (EPI == EPI_RESID) v += rv[i][r];
          if constexpr (OUT_F32)
            reinterpret_cast<float*>(Cv)[(size_t)m * ldc + col] = v;
          else
            reinterpret_cast<uint16_t*>(Cv)[(size_t)m * ldc + col] = f2bf(v);
        }
    }
  }
}

int launch_gemm_tn(const uint16_t* A, int lda, const uint16_t* B, int ldb, const uint16_t* R, int ldr, void* C,
                   int ldc, bool out_f32, int epi, int M, int N, int K, hipStream_t s) {
  if (M <= 0 || N <= 0) return 0;
  if (M % TN_BM || N % TN_BN || K % TN_BK || K <= 0 || lda % 8 || ldb % 8) return -1;
  if (epi != EPI_NONE && epi != EPI_RESID) return -1;
  if (epi == EPI_RESID && (R == nullptr || out_f32)) return -1;
  constexpr int SMEM = 2 * TN_STAGE * 2;  // two stages of two 32 KB images
  const int grid = (M / TN_BM) * (N / TN_BN);
#define XOT_TN(E, F)                                                                                       \
  do {                                                                                                     \
    static bool attr = hipFuncSetAttribute((const void*)gemm_tn_kernel<E, F>,                              \
                                           hipFuncAttributeMaxDynamicSharedMemorySize, SMEM) == hipSuccess; \
    (void)attr;                                                                                            \
    gemm_tn_kernel<E, F><<<grid, 512, SMEM, s>>>(A, lda, B, ldb, R, ldr, C, ldc, M, N, K);                 \
  } while (0)
  if (epi == EPI_RESID)
    XOT_TN(EPI_RESID, false);
  else if (out_f32)
    XOT_TN(EPI_NONE, true);
  else
    XOT_TN(EPI_NONE, false);
#undef XOT_TN
  return 0;
}

}  // namespace xot

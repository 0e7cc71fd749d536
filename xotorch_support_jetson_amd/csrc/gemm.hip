// MFMA GEMMs for the transformer projections:  Y[M,N] = X[M,K] . W[N,K]^T  (nn.Linear / HF layout)
//
//  * gemm_skinny: decode-shaped M <= 128.  Memory-bound on the weight stream, so every weight byte
//    is read exactly once: a workgroup owns 16*NT output columns for ALL M rows and its 4 waves
//    split K; each lane streams 16*KS contiguous bytes per weight row per iteration straight into
//    VGPRs (no LDS round-trip: the W operand is not shared between waves).  The K split is reduced
//    through LDS once at the end, where the fused epilogue runs:
//       EPI_NONE     Y = acc (+bias)
//       EPI_RESID    Y = R + acc (+bias)          (o_proj / down_proj + residual stream)
//       EPI_SILU     Y[:, j] = silu(acc_gate) * acc_up   (gate/up weights interleaved per 16 rows)
//  * gemm_tiled: prefill-shaped M.  128x128x64 LDS tiles, 4 waves in 2x2, register-staged
//    global->LDS copy of tile k+1 overlapped with the MFMAs of tile k (async-STAGE split),
//    padded rows (144 B) so every 16-lane ds_read_b128 group hits 16 distinct bank quads.
//
// Reference parity: replaces the q/k/v/o projections and FeedForward w1/w2/w3 of the torchtune
// layers built in xotorch/inference/torch/models/general_mha.py:77-120 and llm_utils.py:513-522.
#include "common.h"
#include "kernels.h"

namespace xot {

enum { EPI_NONE = 0, EPI_RESID = 1, EPI_SILU = 2 };

template <int MT, int NT, int KS, int EPI, bool OUT_F32>
__global__ __launch_bounds__(256) void gemm_skinny_kernel(const uint16_t* __restrict__ X, int ldx,
                                                          const uint16_t* __restrict__ W, int ldw,
                                                          const uint16_t* __restrict__ bias,
                                                          const uint16_t* __restrict__ R, int ldr,
                                                          void* __restrict__ Yv, int ldy, int M, int K) {
  constexpr int NACC = MT * NT;
  __shared__ f32x4 red[3][NACC][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, c = lane & 15;
  const int n0 = blockIdx.x * 16 * NT;  // first W row of this workgroup
  constexpr int KC = 32 * KS;           // k consumed per iteration by one wave
  const int nchunks = K / KC;

  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const uint16_t* wp[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) wp[j] = W + (size_t)(n0 + 16 * j + c) * ldw + g * 8 * KS;
  const uint16_t* xp[MT];
  bool xok[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int m = 16 * i + c;
    xok[i] = m < M;
    xp[i] = X + (size_t)(xok[i] ? m : 0) * ldx + g * 8 * KS;
  }

  for (int ch = wave; ch < nchunks; ch += 4) {
    const int k0 = ch * KC;
    s16x8 wv[NT][KS], xv[MT][KS];
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int s = 0; s < KS; ++s) wv[j][s] = __builtin_nontemporal_load(reinterpret_cast<const s16x8*>(wp[j] + k0 + 8 * s));
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        s16x8 v = ld16(xp[i] + k0 + 8 * s);
        xv[i][s] = xok[i] ? v : s16x8{0, 0, 0, 0, 0, 0, 0, 0};
      }
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = mfma16(xv[i][s], wv[j][s], acc[i][j]);
  }

  if (wave > 0) {
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) red[wave - 1][i * NT + j][lane] = acc[i][j];
  }
  __syncthreads();
  if (wave != 0) return;
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      acc[i][j] += red[0][i * NT + j][lane];
      acc[i][j] += red[1][i * NT + j][lane];
      acc[i][j] += red[2][i * NT + j][lane];
    }

  if constexpr (EPI == EPI_SILU) {
    // NT == 2: n-tile 0 = gate rows [16b, 16b+16), n-tile 1 = matching up rows
    const int col = blockIdx.x * 16 + c;
    float bg = 0.f, bu = 0.f;
    if (bias != nullptr) {
      bg = bf2f(bias[n0 + c]);
      bu = bf2f(bias[n0 + 16 + c]);
    }
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = 16 * i + 4 * g + r;
        if (m < M) {
          const float v = silu(acc[i][0][r] + bg) * (acc[i][1][r] + bu);
          if constexpr (OUT_F32)
            reinterpret_cast<float*>(Yv)[(size_t)m * ldy + col] = v;
          else
            reinterpret_cast<uint16_t*>(Yv)[(size_t)m * ldy + col] = f2bf(v);
        }
      }
  } else {
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int col = n0 + 16 * j + c;
      const float b = bias != nullptr ? bf2f(bias[col]) : 0.f;
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = 16 * i + 4 * g + r;
          if (m < M) {
            float v = acc[i][j][r] + b;
            if constexpr (EPI == EPI_RESID) v += bf2f(R[(size_t)m * ldr + col]);
            if constexpr (OUT_F32)
              reinterpret_cast<float*>(Yv)[(size_t)m * ldy + col] = v;
            else
              reinterpret_cast<uint16_t*>(Yv)[(size_t)m * ldy + col] = f2bf(v);
          }
        }
    }
  }
}

template <int MT, int NT, int KS, int EPI, bool F32>
static void skinny_launch(const uint16_t* X, int ldx, const uint16_t* W, int ldw, const uint16_t* bias,
                          const uint16_t* R, int ldr, void* Y, int ldy, int M, int N, int K, hipStream_t s) {
  const int grid = N / (16 * NT);
  gemm_skinny_kernel<MT, NT, KS, EPI, F32><<<grid, 256, 0, s>>>(X, ldx, W, ldw, bias, R, ldr, Y, ldy, M, K);
}

template <int EPI, bool F32>
static int skinny_dispatch(const uint16_t* X, int ldx, const uint16_t* W, int ldw, const uint16_t* bias,
                           const uint16_t* R, int ldr, void* Y, int ldy, int M, int N, int K, int nt,
                           hipStream_t s) {
  // returns 0 on success, -1 if the shape is unsupported (caller falls back)
  const int mt = (M + 15) / 16;
  if (EPI == EPI_SILU) nt = 2;
  if (N % (16 * nt) != 0) return -1;
#define XOT_SK(MTV, KSV)                                                                              \
  do {                                                                                                \
    if (K % (32 * KSV) != 0) return -1;                                                               \
    if (nt == 1)                                                                                      \
      skinny_launch<MTV, 1, KSV, EPI, F32>(X, ldx, W, ldw, bias, R, ldr, Y, ldy, M, N, K, s);         \
    else                                                                                              \
      skinny_launch<MTV, 2, KSV, EPI, F32>(X, ldx, W, ldw, bias, R, ldr, Y, ldy, M, N, K, s);         \
    return 0;                                                                                         \
  } while (0)
  if (mt <= 1) XOT_SK(1, 4);
  if (mt <= 2) XOT_SK(2, 4);
  if (mt <= 4) XOT_SK(4, 4);
  if (mt <= 8) XOT_SK(8, 2);
#undef XOT_SK
  return -1;
}

int launch_gemm_skinny(const uint16_t* X, int ldx, const uint16_t* W, int ldw, const uint16_t* bias,
                       const uint16_t* R, int ldr, void* Y, int ldy, bool out_f32, int epi, int M, int N, int K,
                       int nt, hipStream_t s) {
  if (M <= 0) return 0;
  if (epi == EPI_SILU && N % 32 != 0) return -1;
  if (epi == EPI_SILU) return out_f32 ? skinny_dispatch<EPI_SILU, true>(X, ldx, W, ldw, bias, R, ldr, Y, ldy, M, N, K, nt, s)
                                      : skinny_dispatch<EPI_SILU, false>(X, ldx, W, ldw, bias, R, ldr, Y, ldy, M, N, K, nt, s);
  if (epi == EPI_RESID) return skinny_dispatch<EPI_RESID, false>(X, ldx, W, ldw, bias, R, ldr, Y, ldy, M, N, K, nt, s);
  return out_f32 ? skinny_dispatch<EPI_NONE, true>(X, ldx, W, ldw, bias, R, ldr, Y, ldy, M, N, K, nt, s)
                 : skinny_dispatch<EPI_NONE, false>(X, ldx, W, ldw, bias, R, ldr, Y, ldy, M, N, K, nt, s);
}

// ------------------------------------------------------------------------------------ tiled
constexpr int TBM = 128, TBN = 128, TBK = 64, TLD = TBK + 8;  // LDS row = 144 B

template <int EPI, bool OUT_F32>
__global__ __launch_bounds__(256) void gemm_tiled_kernel(const uint16_t* __restrict__ X, int ldx,
                                                         const uint16_t* __restrict__ W, int ldw,
                                                         const uint16_t* __restrict__ bias,
                                                         const uint16_t* __restrict__ R, int ldr,
                                                         void* __restrict__ Yv, int ldy, int M, int N, int K) {
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  uint16_t* As = smem;                      // [2][TBM][TLD]
  uint16_t* Bs = smem + 2 * TBM * TLD;      // [2][TBN][TLD]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c = lane & 15;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = blockIdx.y * TBM, n0 = blockIdx.x * TBN;

  // staging: each thread copies 4 x 16 B of A and 4 x 16 B of B per K-tile
  // chunk id q = tid + 256*i  -> row = q >> 3, col8 = (q & 7) * 8
  s16x8 ra[4], rb[4];
  auto gload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int q = tid + 256 * i, row = q >> 3, col = (q & 7) * 8;
      const int gm = m0 + row, gn = n0 + row;
      ra[i] = gm < M ? ld16(X + (size_t)gm * ldx + k0 + col) : s16x8{0, 0, 0, 0, 0, 0, 0, 0};
      rb[i] = gn < N ? ld16(W + (size_t)gn * ldw + k0 + col) : s16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
  };
  auto swrite = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int q = tid + 256 * i, row = q >> 3, col = (q & 7) * 8;
      st16(As + (buf * TBM + row) * TLD + col, ra[i]);
      st16(Bs + (buf * TBN + row) * TLD + col, rb[i]);
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = K / TBK;
  gload(0);
  swrite(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) gload((kt + 1) * TBK);  // issue early, land under the MFMAs
#pragma unroll
    for (int s = 0; s < TBK / 32; ++s) {
      s16x8 af[4], bf[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = ld16(As + (buf * TBM + wm * 64 + 16 * i + c) * TLD + 32 * s + 8 * g);
#pragma unroll
      for (int j = 0; j < 4; ++j) bf[j] = ld16(Bs + (buf * TBN + wn * 64 + 16 * j + c) * TLD + 32 * s + 8 * g);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(af[i], bf[j], acc[i][j]);
    }
    if (kt + 1 < nk) swrite(buf ^ 1);  // other buffer: last read one iteration ago (barrier below)
    __syncthreads();
  }

#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = n0 + wn * 64 + 16 * j + c;
    if (col >= N) continue;
    const float b = bias != nullptr ? bf2f(bias[col]) : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 64 + 16 * i + 4 * g + r;
        if (m < M) {
          float v = acc[i][j][r] + b;
          if constexpr (EPI == EPI_RESID) v += bf2f(R[(size_t)m * ldr + col]);
          if constexpr (OUT_F32)
            reinterpret_cast<float*>(Yv)[(size_t)m * ldy + col] = v;
          else
            reinterpret_cast<uint16_t*>(Yv)[(size_t)m * ldy + col] = f2bf(v);
        }
      }
  }
}

int launch_gemm_tiled(const uint16_t* X, int ldx, const uint16_t* W, int ldw, const uint16_t* bias,
                      const uint16_t* R, int ldr, void* Y, int ldy, bool out_f32, int epi, int M, int N, int K,
                      hipStream_t s) {
  if (M <= 0) return 0;
  if (K % TBK != 0 || epi == EPI_SILU) return -1;
  dim3 grid((N + TBN - 1) / TBN, (M + TBM - 1) / TBM);
  const size_t lds = (size_t)2 * (TBM + TBN) * TLD * sizeof(uint16_t);
  if (epi == EPI_RESID) {
    if (out_f32) return -1;
    hipLaunchKernelGGL((gemm_tiled_kernel<EPI_RESID, false>), grid, dim3(256), lds, s, X, ldx, W, ldw, bias, R,
                       ldr, Y, ldy, M, N, K);
  } else if (out_f32) {
    hipLaunchKernelGGL((gemm_tiled_kernel<EPI_NONE, true>), grid, dim3(256), lds, s, X, ldx, W, ldw, bias, R, ldr,
                       Y, ldy, M, N, K);
  } else {
    hipLaunchKernelGGL((gemm_tiled_kernel<EPI_NONE, false>), grid, dim3(256), lds, s, X, ldx, W, ldw, bias, R,
                       ldr, Y, ldy, M, N, K);
  }
  return 0;
}

}  // namespace xot

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
#include "gemm_common.h"
#include "kernels.h"

namespace xot {

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

  if constexpr (EPI == EPI_SILU && NT == 2) {
    // n-tile 0 = gate rows [16b, 16b+16), n-tile 1 = matching up rows
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
  } else if constexpr (EPI != EPI_SILU) {
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

// ------------------------------------------------------------------------------------ stream
// Decode GEMM v2.  Workgroup = 4 waves side by side along N (wave w owns W rows
// [n0 + 16*NTW*w, +16*NTW)), all M rows (<= 16*MT), K range [blockIdx.y*kper, +kper).
// Per k-chunk (KC = 32*KS):
//   X[:, chunk]  : cooperatively register-staged into an XOR-swizzled LDS double buffer
//                  (physical 16-B slot = logical ^ (row & (CPR-1))) -> the 16-lane ds_read_b128
//                  groups of the A-fragment reads hit 16 distinct bank quads
//   W rows       : streamed once, straight to VGPRs, two chunks in flight (prefetch depth 2)
// MFMA k-order is permuted per lane group (group g owns k in [8*KS*g, 8*KS*(g+1)) of the chunk)
// so each lane reads 16*KS contiguous bytes of its weight row per chunk.
// SPLIT: fp32 partial slabs ws[blockIdx.y][M][N], finished by splitk_reduce_kernel or by the consumer's fused reduce
// (a last-arriver combine inside the launch measured no faster at batch 1 and 3 % slower at 512: removed in round 6).
// MOE = 3: batched GEMM (per-head projections of MLA): blockIdx.z = problem e, weight W[e], A rows X + e*xbat,
// output Y + e*ybat (element offsets; row strides ldx / ldy shared), all M rows.
// MOE = 1 / 2: grouped (mixture-of-experts) GEMM.  blockIdx.z = expert e with weight W[e]
// ([E][N][K], same layout per expert) and rows moe_off[e] .. moe_off[e+1] of the expert-sorted slot
// order; MOE = 1 reads A in slot order, MOE = 2 gathers A row moe_gather[slot] (token rows).  Output
// rows are slots.  Row blocks past an expert's count exit at once, so the grid can be sized for the
// worst case on the host and the launch stays graph-capturable (no host sync on the routing).
// W8: weight-only FP8 (OCP e4m3, per-output-row fp32 scale `wscale`): pre-shuffled tiles of 16 rows x 128 k
// as [N/16][K/128][2][lane][16 B], the 16 bytes of lane (g, c) in half h being row c, k 64 h + 8 g .. +8
// (bytes 0-7) and 64 h + 32 + 8 g .. +8 (bytes 8-15): one 1 KB wave load carries two MFMA k-steps, half
// the bytes of the bf16 layout.  v_cvt_scalef32_pk_bf16_fp8 widens each fragment just before its MFMAs;
// the row scale is applied to the fp32 accumulators (so split-K slabs are already scaled).
template <int MT, int NTW, int KS, int EPI, bool OUT_F32, bool SPLIT, bool WSHUF, int OCC, int MOE, bool W8 = false,
          int NORM = 0, bool MERGE = false>
__global__ __launch_bounds__(256, OCC) void gemm_stream_kernel(const uint16_t* __restrict__ X, int ldx,
                                                             const uint16_t* __restrict__ W, int ldw,
                                                             const uint16_t* __restrict__ bias,
                                                             const uint16_t* __restrict__ R, int ldr,
                                                             void* __restrict__ Yv, int ldy,
                                                             float* __restrict__ ws, int M, int N, int kper,
                                                             int mblocks, const int* __restrict__ moe_off,
                                                             const int* __restrict__ moe_gather,
                                                             int* __restrict__ tickets, long ysplit,
                                                             const float* __restrict__ wscale, long xbat,
                                                             long ybat, NormPro np) {
  constexpr int KC = 32 * KS;
  static_assert(!W8 || (WSHUF && (KS == 4 || KS == 8) && MOE == 0),
                "FP8 weights: pre-shuffled 128- or 256-deep chunks, dense GEMM");
  constexpr int CPR = KC / 8;  // 16-B chunks per row per k-chunk
  constexpr int NTH = 256;
  constexpr int ROWS = 16 * MT;
  constexpr int XPT = ROWS * CPR / NTH;  // staging chunks per thread
  static_assert(XPT >= 1, "tile too small for 256 threads");
  static_assert(MOE == 0 || !SPLIT, "grouped GEMM runs without split-K");
  // X double buffer in dynamic LDS (2 x ROWS x KC bf16)
  extern __shared__ __attribute__((aligned(16))) uint16_t xs_raw[];
  auto xs = reinterpret_cast<uint16_t(*)[ROWS * KC]>(xs_raw);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int wrow = 0;
  const int g = lane >> 4, c = lane & 15;
  // M-blocking (M > ROWS): blockIdx.x = (column tile, row block).  The row blocks of one column tile
  // get ids 8 apart, i.e. the same XCD under round-robin dispatch, and run together: the weight tile
  // comes from HBM once and from that XCD's L2 for the other row blocks.
  int bt = blockIdx.x, mb = 0;
  if (mblocks > 1) {
    const int ntiles = N / (64 * NTW);
    if ((ntiles & 7) == 0) {
      const int grp = 8 * mblocks, q = bt / grp, rem = bt % grp;
      mb = rem >> 3;
      bt = 8 * q + (rem & 7);
    } else {
      mb = bt % mblocks;
      bt /= mblocks;
    }
  }
  int row0 = 0;  // first output row of this launch's row range
  if constexpr (MOE == 3) {  // batched: problem e = blockIdx.z has W[e], X + e * xbat, Y + e * ybat
    const int e = blockIdx.z;
    W += (size_t)e * N * ldw;
    X += (size_t)e * xbat;
    if constexpr (OUT_F32)
      Yv = reinterpret_cast<float*>(Yv) + (size_t)e * ybat;
    else
      Yv = reinterpret_cast<uint16_t*>(Yv) + (size_t)e * ybat;
  }
  if constexpr (MOE == 1 || MOE == 2) {
    const int e = blockIdx.z;
    row0 = moe_off[e];
    M = moe_off[e + 1] - row0;  // this expert's rows
    W += (size_t)e * N * ldw;
    if (mb * ROWS >= M) return;  // uniform over the workgroup, before any barrier
  }
  // grouped GEMM split over K: K slice blockIdx.y writes its own fp32 slab of Y (ysplit elements apart),
  // summed by the consumer (moe_combine_kernel)
  if constexpr (MOE == 1 || MOE == 2) {
    if (ysplit != 0) Yv = reinterpret_cast<float*>(Yv) + (size_t)blockIdx.y * ysplit;
  }
  const int Mtot = M, m_base = mb * ROWS;
  M = min(ROWS, Mtot - m_base);
  if constexpr (MOE != 2) X += (size_t)(row0 + m_base) * ldx;
  if constexpr (EPI == EPI_RESID) R += (size_t)(row0 + m_base) * ldr;
  if constexpr (OUT_F32)
    Yv = reinterpret_cast<float*>(Yv) + (size_t)(row0 + m_base) * ldy;
  else
    Yv = reinterpret_cast<uint16_t*>(Yv) + (size_t)(row0 + m_base) * ldy;
  const int n0 = bt * (64 * NTW) + wave * 16 * NTW;
  const int kb = blockIdx.y * kper;
  const int nch = kper / KC;

  // W pointers.  Row-major: lane (g, c) streams row n0+16j+c, k in [8*KS*g, 8*KS*(g+1)) of each chunk.
  // Pre-shuffled (WSHUF, KS == 4): tiles [N/16][K/128][s][lane][8] so instruction s of a wave reads
  // 1 KB of contiguous memory holding the MFMA B fragments of k [32s, 32s+32) in natural order (lane
  // (g, c): row c, k 32s+8g..+8; see ops.weights_layout.shuffle_for_stream).
  const uint16_t* wp[NTW];
  constexpr int WSTEP = WSHUF ? 16 * KC : KC;  // elements between consecutive chunks of one lane
#pragma unroll
  for (int j = 0; j < NTW; ++j) {
    if constexpr (W8)  // byte pointer carried as uint16_t*: chunks are 2 KB = 1024 "elements" apart
      wp[j] = reinterpret_cast<const uint16_t*>(reinterpret_cast<const uint8_t*>(W) +
                                                ((size_t)((n0 >> 4) + j) * (ldw / KC) + kb / KC) * (16 * KC) + lane * 16);
    else if constexpr (WSHUF)
      wp[j] = W + ((size_t)((n0 >> 4) + j) * (ldw / KC) + kb / KC) * (16 * KC) + lane * 8;
    else
      wp[j] = W + (size_t)(n0 + 16 * j + c) * ldw + kb + g * 8 * KS;
  }

  // staging geometry of this thread's XPT chunks, recomputed on use (keeps VGPRs for the pipeline):
  // chunk q = tid + NTH*i -> row q / CPR, logical 16-B slot q % CPR
  const uint16_t* xbase = X + kb;
  int srow[MOE == 2 ? XPT : 1];  // gathered source rows of this thread's staging chunks
  if constexpr (MOE == 2) {
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int row = (tid + NTH * i) / CPR;
      srow[i] = row < M ? moe_gather[row0 + m_base + row] : 0;
    }
  }
  auto xload = [&](s16x8 (&xr)[XPT], int ch) {
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int q = tid + NTH * i, row = q / CPR, cc = q % CPR;
      const bool ok = row < M;
      const int src = MOE == 2 ? srow[i] : (ok ? row : 0);
      s16x8 v = ld16(xbase + (size_t)src * ldx + ch * KC + cc * 8);
      xr[i] = ok ? v : s16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
  };
  auto xstore = [&](const s16x8 (&xr)[XPT], int buf) {
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int q = tid + NTH * i, row = q / CPR, cc = q % CPR;
      st16(&xs[buf][row * KC + ((cc ^ (row & (CPR - 1))) * 8)], xr[i]);
    }
  };
  auto wload = [&](s16x8 (&wr)[NTW][KS], int ch) {
#pragma unroll
    for (int j = 0; j < NTW; ++j)
#pragma unroll
      for (int s = 0; s < (W8 ? KS / 2 : KS); ++s)
        wr[j][s] = __builtin_nontemporal_load(reinterpret_cast<const s16x8*>(
            W8 ? wp[j] + ch * (8 * KC) + 512 * s : wp[j] + ch * WSTEP + (WSHUF ? 512 * s : 8 * s)));
  };
  // B fragment of k-step s for column tile j (W8: widen 8 e4m3 values of the raw 16-byte load)
  auto bfrag = [&](const s16x8 (&wr)[NTW][KS], int j, int s) -> s16x8 {
    if constexpr (W8) {
      const u32x4 raw = __builtin_bit_cast(u32x4, wr[j][s >> 1]);
      const uint32_t lo = raw[(s & 1) * 2], hi = raw[(s & 1) * 2 + 1];
      u32x4 o;
      o[0] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(lo, 1.0f, false));
      o[1] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(lo, 1.0f, true));
      o[2] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(hi, 1.0f, false));
      o[3] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(hi, 1.0f, true));
      return __builtin_bit_cast(s16x8, o);
    } else {
      return wr[j][s];
    }
  };

  f32x4 acc[MT][NTW];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NTW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // nch >= 1: prologue loads chunks 0 and 1.  An odd chunk count (grouped GEMMs over K = 128 * odd, e.g.
  // DeepSeek-V2-Lite's 1408-wide experts) re-loads the last chunk where a pair would run past it (the
  // loads stay unconditional) and finishes with a single-chunk tail.
  const int last = nch - 1;
  s16x8 wa[NTW][KS], wb[NTW][KS];
  if constexpr (NORM > 0 || MERGE) {
  static_assert(MT == 1 && MOE == 0 && !W8 && WSHUF, "row prologue: one row, pre-shuffled bf16 weights");
  uint16_t* x1 = xs_raw;  // this workgroup's K slice of the input row, [kper] bf16
  wload(wa, 0);
  wload(wb, min(1, last));
  if constexpr (MERGE) {
    // split-KV decode attention merge (attn_decode_reduce_kernel's arithmetic, in its order) for the heads of
    // this workgroup's K slice: o = sum_p 2^(m_p - M) o_p / sum_p 2^(m_p - M) l_p over the row's partitions
    const int npages = (max(np.ctx[0], 0) + 63) / 64;
    int npart = (npages + np.ppp - 1) / np.ppp;
    npart = npart < 1 ? 1 : (npart > np.nparts ? np.nparts : npart);
    constexpr int NPM = 8;  // partitions whose loads are all requested before use (more: a second, per-element loop)
    for (int e0 = 4 * tid; e0 < kper; e0 += 4 * NTH) {  // 4 consecutive elements of one head per thread
      const int k = kb + e0, hd = k / np.dh, d = k - hd * np.dh;
      const size_t base = (size_t)hd * np.nparts;
      float o4[4];
      if (npart <= NPM) {
        f32x2_t mv[NPM];
        f32x4 ov[NPM];
#pragma unroll
        for (int q = 0; q < NPM; ++q)
          if (q < npart) {
            mv[q] = *reinterpret_cast<const f32x2_t*>(np.ml + (base + q) * 2);
            ov[q] = *reinterpret_cast<const f32x4*>(np.mo + (base + q) * np.dh + d);
          }
        float M = -1e30f;
#pragma unroll
        for (int q = 0; q < NPM; ++q)
          if (q < npart) M = fmaxf(M, mv[q][0]);
        float L = 0.f, O[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int q = 0; q < NPM; ++q)
          if (q < npart) {
            const float f = exp2f(mv[q][0] - M);
            L += mv[q][1] * f;
#pragma unroll
            for (int j = 0; j < 4; ++j) O[j] += ov[q][j] * f;
          }
#pragma unroll
        for (int j = 0; j < 4; ++j) o4[j] = L > 0.f ? O[j] / L : 0.f;
      } else {
        float M = -1e30f;
        for (int q = 0; q < npart; ++q) M = fmaxf(M, np.ml[(base + q) * 2]);
        float L = 0.f, O[4] = {0.f, 0.f, 0.f, 0.f};
        for (int q = 0; q < npart; ++q) {
          const float f = exp2f(np.ml[(base + q) * 2] - M);
          L += np.ml[(base + q) * 2 + 1] * f;
#pragma unroll
          for (int j = 0; j < 4; ++j) O[j] += np.mo[(base + q) * np.dh + d + j] * f;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) o4[j] = L > 0.f ? O[j] / L : 0.f;
      }
      *reinterpret_cast<s16x4*>(x1 + e0) =
          s16x4{(short)f2bf(o4[0]), (short)f2bf(o4[1]), (short)f2bf(o4[2]), (short)f2bf(o4[3])};
    }
  } else {
    // RMSNorm prologue (one input row; NORM = 16-B chunks of the row per thread): the first two weight chunks,
    // then every residual / bias / norm-weight load and the first SMAX slabs are requested before any is used,
    // so the chain is one L2 round trip per SMAX slabs (the producer just wrote them), one wave reduction and two
    // barriers, under the weight stream's own HBM latency.  Same arithmetic and reduction order as
    // splitk_resid_rmsnorm_kernel<*, *, 256>: the row is bitwise the one the unfused pair gives.
    constexpr int PM = NORM, SMAX = NORM >= 4 ? 2 : 8;  // slabs per round trip (registers: PM x SMAX x 8)
    __shared__ float nred[NTH / 64];
    const int nchunk = np.D >> 3, c0 = kb >> 3, c1 = (kb + kper) >> 3;
    const bool wg0 = blockIdx.x == 0 && blockIdx.y == 0;
    s16x8 ha[PM], ba[PM], la[PM];
    f32x4 p[PM][SMAX][2];
    // slabs s0 .. s0 + SMAX - 1 of this thread's chunks (all requested before any is added)
    auto slabs = [&](int s0) {
#pragma unroll
      for (int i = 0; i < PM; ++i) {
        const int cc = tid + NTH * i;
        if (cc < nchunk) {
#pragma unroll
          for (int sl = 0; sl < SMAX; ++sl)
            if (s0 + sl < np.S) {
              const float* sp = np.ws + (s0 + sl) * np.sstride + cc * 8;
              p[i][sl][0] = *reinterpret_cast<const f32x4*>(sp);
              p[i][sl][1] = *reinterpret_cast<const f32x4*>(sp + 4);
            }
        }
      }
    };
#pragma unroll
    for (int i = 0; i < PM; ++i) {
      const int cc = tid + NTH * i;
      if (cc < nchunk) {
        ha[i] = ld16(np.h + cc * 8);
        if (np.bias != nullptr) ba[i] = ld16(np.bias + cc * 8);
        if (cc >= c0 && cc < c1) la[i] = ld16(np.lnw + cc * 8);
      }
    }
    slabs(0);
    float v[PM][8];
#pragma unroll
    for (int i = 0; i < PM; ++i) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[i][j] = bf2f(ha[i][j]);
      if (np.bias != nullptr) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] += bf2f(ba[i][j]);
      }
    }
    for (int s0 = 0; s0 < np.S; s0 += SMAX) {  // one L2 round trip per SMAX slabs
      if (s0 > 0) slabs(s0);
#pragma unroll
      for (int i = 0; i < PM; ++i)
#pragma unroll
        for (int sl = 0; sl < SMAX; ++sl)
          if (s0 + sl < np.S) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              v[i][j] += p[i][sl][0][j];
              v[i][4 + j] += p[i][sl][1][j];
            }
          }
    }
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < PM; ++i) {
      const int cc = tid + NTH * i;
      if (cc < nchunk) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          ha[i][j] = (short)f2bf(v[i][j]);
          const float r = bf2f(ha[i][j]);
          ss += r * r;
        }
        if (wg0) st16(np.hout + cc * 8, ha[i]);
      }
    }
    ss = wave_sum(ss);
    if (lane == 0) nred[wave] = ss;
    __syncthreads();
    ss = 0.f;
#pragma unroll
    for (int k = 0; k < NTH / 64; ++k) ss += nred[k];
    const float inv = rsqrtf(ss / (float)np.D + np.eps);
#pragma unroll
    for (int i = 0; i < PM; ++i) {
      const int cc = tid + NTH * i;
      if (cc < nchunk && cc >= c0 && cc < c1) {
        s16x8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = (short)f2bf(bf2f(ha[i][j]) * inv * bf2f(la[i][j]));
        st16(x1 + (cc - c0) * 8, o);
      }
    }
  }
    __syncthreads();
    // row 0 is the only real row: its A fragments come from the slice (natural k order of the pre-shuffled
    // layout: lane group g holds k 32 s + 8 g .. +8), the other 15 MFMA rows are zero
    auto compute_n = [&](const s16x8 (&wr)[NTW][KS], int ch) {
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const s16x8 a = c == 0 ? ld16(x1 + ch * KC + (4 * s + g) * 8) : s16x8{0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int j = 0; j < NTW; ++j) acc[0][j] = mfma16(a, wr[j][s], acc[0][j]);
      }
    };
    int ch = 0;
    for (; ch + 2 < nch; ch += 2) {
      compute_n(wa, ch);
      wload(wa, ch + 2);
      compute_n(wb, ch + 1);
      wload(wb, min(ch + 3, last));
    }
    compute_n(wa, ch);
    if (!(nch & 1)) compute_n(wb, ch + 1);
  } else {
  s16x8 xr[XPT];
  xload(xr, 0);
  wload(wa, 0);
  xstore(xr, 0);
  xload(xr, min(1, last));
  wload(wb, min(1, last));
  __syncthreads();

  // A fragments are software-pipelined LDPF reads ahead of their MFMAs; the scheduling fences keep
  // the compiler from hoisting the whole chunk's LDS reads (which costs 100+ VGPRs and spills).
  constexpr int LDPF = 4;
  auto compute = [&](const s16x8 (&wr)[NTW][KS], int buf) {
    const uint16_t* xb = &xs[buf][0];
    auto afrag = [&](int t) {
      const int s = t / MT, i = t % MT;
      const int row = wrow + 16 * i + c;
      // row-major W: lane group g owns k [8*KS*g, +8*KS) of the chunk; pre-shuffled W: natural MFMA order
      const int phys = (WSHUF ? (4 * s + g) : (g * KS + s)) ^ (row & (CPR - 1));
      return ld16(xb + row * KC + phys * 8);
    };
    s16x8 a[LDPF];
#pragma unroll
    for (int t = 0; t < LDPF; ++t) a[t] = afrag(t);
#pragma unroll
    for (int t = 0; t < KS * MT; ++t) {
      const int s = t / MT, i = t % MT;
      const s16x8 cur = a[t % LDPF];
      if (t + LDPF < KS * MT) a[t % LDPF] = afrag(t + LDPF);
#pragma unroll
      for (int j = 0; j < NTW; ++j) acc[i][j] = mfma16(cur, bfrag(wr, j, s), acc[i][j]);
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // Steady state: two chunks per trip (static register double buffer), every load unconditional so
  // hipcc's waitcnt pass keeps counted vmcnt(N) waits across the back-edge instead of draining to 0.
  int ch = 0;
  for (; ch + 2 < nch; ch += 2) {
    compute(wa, 0);
    xstore(xr, 1);
    __syncthreads();
    xload(xr, ch + 2);
    wload(wa, ch + 2);
    compute(wb, 1);
    xstore(xr, 0);
    __syncthreads();
    xload(xr, min(ch + 3, last));
    wload(wb, min(ch + 3, last));
  }
  if (nch & 1) {
    compute(wa, 0);  // tail: chunk nch-1 (wa, buf 0)
  } else {
    // tail: chunks nch-2 (wa, buf 0) and nch-1 (wb / xr)
    compute(wa, 0);
    xstore(xr, 1);
    __syncthreads();
    compute(wb, 1);
  }
  }  // !NORM

  if constexpr (W8) {
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
      const float sc = wscale[n0 + 16 * j + c];
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[i][j][r] *= sc;
    }
  }

  if constexpr (SPLIT) {
    float* slab = ws + ((size_t)blockIdx.y * Mtot + m_base) * N;
#pragma unroll
    for (int j = 0; j < NTW; ++j)
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = wrow + 16 * i + 4 * g + r;
          if (m < M) slab[(size_t)m * N + n0 + 16 * j + c] = acc[i][j][r];
        }
  } else if constexpr (EPI == EPI_SILU && NTW >= 2) {
#pragma unroll
    for (int p = 0; p < NTW / 2; ++p) {  // pair (gate tile 2p, up tile 2p+1) -> 16 output columns
      const int col = (n0 >> 1) + 16 * p + c;
      float bg = 0.f, bu = 0.f;
      if (bias != nullptr) {
        bg = bf2f(bias[n0 + 32 * p + c]);
        bu = bf2f(bias[n0 + 32 * p + 16 + c]);
      }
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = wrow + 16 * i + 4 * g + r;
          if (m < M) {
            const float v = silu(acc[i][2 * p][r] + bg) * (acc[i][2 * p + 1][r] + bu);
            if constexpr (OUT_F32)
              reinterpret_cast<float*>(Yv)[(size_t)m * ldy + col] = v;
            else
              reinterpret_cast<uint16_t*>(Yv)[(size_t)m * ldy + col] = f2bf(v);
          }
        }
    }
  } else if constexpr (EPI != EPI_SILU) {
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
      const int col = n0 + 16 * j + c;
      const float b = bias != nullptr ? bf2f(bias[col]) : 0.f;
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = wrow + 16 * i + 4 * g + r;
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

template <int MT, int NTW, int KS, int EPI, bool F32, bool WSH, bool W8 = false>
static void stream_launch(const uint16_t* X, int ldx, const uint16_t* W, int ldw, const uint16_t* bias,
                          const uint16_t* R, int ldr, void* Y, int ldy, float* ws, int M, int N, int K, int S,
                          bool reduce, hipStream_t st, const float* wscale = nullptr) {
  // occupancy request: 2 workgroups/CU while the register budget allows it (FP8 weights need a few more
  // registers for the widened fragments)
  constexpr int OCC = (MT * NTW >= (W8 ? 16 : 32)) ? 1 : 2;
  constexpr int SMEM = 2 * 16 * MT * 32 * KS * 2;
  const int mblocks = (M + 16 * MT - 1) / (16 * MT);
  dim3 grid(N / (64 * NTW) * mblocks, S);
  const int kper = K / S;
  if (S == 1) {
    auto kern = gemm_stream_kernel<MT, NTW, KS, EPI, F32, false, WSH, OCC, 0, W8>;
    if constexpr (SMEM > 65536) {
      static bool attr = (hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM) ==
                          hipSuccess);
      (void)attr;
    }
    kern<<<grid, 256, SMEM, st>>>(X, ldx, W, ldw, bias, R, ldr, Y, ldy, nullptr, M, N, kper, mblocks, nullptr, nullptr,
                                  nullptr, 0L, wscale, 0L, 0L, NormPro{});
  } else {
    auto kern = gemm_stream_kernel<MT, NTW, KS, EPI, F32, true, WSH, OCC, 0, W8>;
    if constexpr (SMEM > 65536) {
      static bool attr = (hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM) ==
                          hipSuccess);
      (void)attr;
    }
    kern<<<grid, 256, SMEM, st>>>(X, ldx, W, ldw, bias, R, ldr, Y, ldy, ws, M, N, kper, mblocks, nullptr, nullptr,
                                  nullptr, 0L, wscale, 0L, 0L, NormPro{});
    if (!reduce) return;  // slabs left for the consumer
    const int ncol = EPI == EPI_SILU ? N / 2 : N;
    long chunks = (long)M * (ncol / 8);
    int blocks = (int)((chunks + 255) / 256);
    if (blocks > 2048) blocks = 2048;
    splitk_reduce_kernel<EPI, F32><<<blocks, 256, 0, st>>>(ws, S, M, N, bias, R, ldr, Y, ldy);
  }
}

template <int EPI, bool F32>
static int stream_dispatch(const uint16_t* X, int ldx, const uint16_t* W, int ldw, const uint16_t* bias,
                           const uint16_t* R, int ldr, void* Y, int ldy, float* ws, long ws_elems, int M, int N,
                           int K, int ntw, int S, bool wshuf, bool reduce, hipStream_t st) {
  if (EPI == EPI_SILU && ntw == 1) ntw = 2;
  if (ntw != 1 && ntw != 2 && ntw != 4) return -1;
  const int mt = (M + 15) / 16;
  if (ntw == 4 && mt <= 2) ntw = 2;
  if (N % (64 * ntw) != 0 || S < 1) return -1;
  const int KS = 4;
  if (K % (S * 32 * KS) != 0) return -1;  // whole 128-deep k-chunks per workgroup (odd counts: single tail)
  if (S > 1 && (ws == nullptr || ws_elems < (long)S * M * N)) return -1;
  if (EPI == EPI_SILU && N % 32 != 0) return -1;
  if (wshuf && (KS != 4 || K % 128 != 0)) return -1;
#define XOT_ST2(MTV, KSV, WSH)                                                                              \
  do {                                                                                                      \
    if (ntw == 1 && EPI != EPI_SILU)                                                                        \
      stream_launch<MTV, 1, KSV, EPI, F32, WSH>(X, ldx, W, ldw, bias, R, ldr, Y, ldy, ws, M, N, K, S, reduce, st);  \
    else if (ntw == 4 && MTV >= 4 && MTV <= 8)                                                                    \
      stream_launch<MTV, 4, KSV, EPI, F32, WSH>(X, ldx, W, ldw, bias, R, ldr, Y, ldy, ws, M, N, K, S, reduce, st);  \
    else                                                                                                    \
      stream_launch<MTV, 2, KSV, EPI, F32, WSH>(X, ldx, W, ldw, bias, R, ldr, Y, ldy, ws, M, N, K, S, reduce, st);  \
    return 0;                                                                                               \
  } while (0)
#define XOT_ST(MTV, KSV)                  \
  do {                                    \
    if (wshuf) XOT_ST2(MTV, KSV, true);   \
    XOT_ST2(MTV, KSV, false);             \
  } while (0)
  if (mt <= 1) XOT_ST(1, 4);
  if (mt <= 2) XOT_ST(2, 4);
  if (mt <= 4) XOT_ST(4, 4);
  if (mt <= 8) XOT_ST(8, 4);
  // M > 128: 128-row blocks; the blocks of one column tile run on one XCD together (see the kernel).
  // (256-row tiles -- MT = 16, or 8 waves as 2 row halves x 4 column groups -- need > 256 registers
  // per lane at this pipeline depth and spill; both measured slower than the M-blocked 128-row tile.)
  XOT_ST(8, 4);
#undef XOT_ST
#undef XOT_ST2
  return -1;
}

// ------------------------------------------------------------------------------------ batched (MLA heads)
template <int MT, bool F32>
static void batched_launch(const uint16_t* X, int ldx, long xbat, const uint16_t* W, void* Y, int ldy, long ybat,
                           int B, int M, int N, int K, hipStream_t st) {
  constexpr int NTW = 2, KS = 4;
  constexpr int OCC = (MT * NTW >= 32) ? 1 : 2;
  constexpr int SMEM = 2 * 16 * MT * 32 * KS * 2;
  const int mblocks = (M + 16 * MT - 1) / (16 * MT);
  dim3 grid(N / (64 * NTW) * mblocks, 1, B);
  gemm_stream_kernel<MT, NTW, KS, EPI_NONE, F32, false, true, OCC, 3><<<grid, 256, SMEM, st>>>(
      X, ldx, W, K, nullptr, nullptr, 0, Y, ldy, nullptr, M, N, K, mblocks, nullptr, nullptr, nullptr, 0L, nullptr,
      xbat, ybat, NormPro{});
}

// B independent GEMMs Y_e[M, N] = X_e[M, K] . W_e[N, K]^T on pre-shuffled weights W [B][N][K]
int launch_gemm_batched(const uint16_t* X, int ldx, long xbat, const uint16_t* W, void* Y, int ldy, long ybat,
                        bool out_f32, int B, int M, int N, int K, hipStream_t s) {
  if (M <= 0 || B <= 0) return 0;
  if (N % 128 != 0 || K % 128 != 0) return -1;
  const int mt = (M + 15) / 16;
#define XOT_BAT(MTV)                                                                                   \
  do {                                                                                                 \
    if (out_f32) batched_launch<MTV, true>(X, ldx, xbat, W, Y, ldy, ybat, B, M, N, K, s);              \
    else batched_launch<MTV, false>(X, ldx, xbat, W, Y, ldy, ybat, B, M, N, K, s);                     \
    return 0;                                                                                          \
  } while (0)
  // the widest row tile that still gives the 256 CUs a workgroup each (decode: M ~ 256 rows, B heads)
  auto wgs = [&](int m) { return (long)(N / 128) * ((M + 16 * m - 1) / (16 * m)) * B; };
  if (mt <= 1) XOT_BAT(1);
  if (mt <= 4) XOT_BAT(4);
  if (wgs(8) >= 256) XOT_BAT(8);
  if (wgs(4) >= 256) XOT_BAT(4);
  XOT_BAT(1);
#undef XOT_BAT
}

// ------------------------------------------------------------------------------------ grouped (MoE)
template <int MT, int EPI, bool F32, bool WSH, int MOE>
static void moe_launch(const uint16_t* X, int ldx, const uint16_t* W, void* Y, int ldy, const int* off,
                       const int* gather, int E, int max_rows, int N, int K, int S, long ysplit, hipStream_t st) {
  constexpr int NTW = 2, KS = 4;
  constexpr int OCC = (MT * NTW >= 32) ? 1 : 2;
  constexpr int SMEM = 2 * 16 * MT * 32 * KS * 2;
  const int mblocks = (max_rows + 16 * MT - 1) / (16 * MT);
  dim3 grid(N / (64 * NTW) * mblocks, S, E);
  gemm_stream_kernel<MT, NTW, KS, EPI, F32, false, WSH, OCC, MOE><<<grid, 256, SMEM, st>>>(
      X, ldx, W, K, nullptr, nullptr, 0, Y, ldy, nullptr, max_rows, N, K / S, mblocks, off, gather, nullptr,
      S > 1 ? ysplit : 0L, nullptr, 0L, 0L, NormPro{});
}

template <int EPI, bool F32, bool WSH, int MOE>
static void moe_mt(const uint16_t* X, int ldx, const uint16_t* W, void* Y, int ldy, const int* off,
                   const int* gather, int E, int max_rows, int N, int K, int S, long ysplit, hipStream_t st) {
  if (max_rows <= 16)
    moe_launch<1, EPI, F32, WSH, MOE>(X, ldx, W, Y, ldy, off, gather, E, max_rows, N, K, S, ysplit, st);
  else if (max_rows <= 64)
    moe_launch<4, EPI, F32, WSH, MOE>(X, ldx, W, Y, ldy, off, gather, E, max_rows, N, K, S, ysplit, st);
  else
    moe_launch<8, EPI, F32, WSH, MOE>(X, ldx, W, Y, ldy, off, gather, E, max_rows, N, K, S, ysplit, st);
}

int launch_gemm_moe(const uint16_t* X, int ldx, const uint16_t* W, void* Y, int ldy, bool out_f32, int epi,
                    const int* off, const int* gather, int E, int max_rows, int N, int K, bool wshuf, int S,
                    long ysplit, hipStream_t s) {
  if (max_rows <= 0) return 0;
  if (N % 128 != 0 || S < 1 || K % (128 * S) != 0) return -1;
  if (epi != EPI_NONE && epi != EPI_SILU) return -1;
  if (epi == EPI_SILU && out_f32) return -1;
  if (S > 1 && (epi != EPI_NONE || !out_f32)) return -1;  // K slices write fp32 partial slabs
#define XOT_MOE(EPIV, F32V)                                                                                     \
  do {                                                                                                          \
    if (wshuf) {                                                                                                \
      if (gather) moe_mt<EPIV, F32V, true, 2>(X, ldx, W, Y, ldy, off, gather, E, max_rows, N, K, S, ysplit, s);  \
      else moe_mt<EPIV, F32V, true, 1>(X, ldx, W, Y, ldy, off, gather, E, max_rows, N, K, S, ysplit, s);         \
    } else {                                                                                                    \
      if (gather) moe_mt<EPIV, F32V, false, 2>(X, ldx, W, Y, ldy, off, gather, E, max_rows, N, K, S, ysplit, s); \
      else moe_mt<EPIV, F32V, false, 1>(X, ldx, W, Y, ldy, off, gather, E, max_rows, N, K, S, ysplit, s);        \
    }                                                                                                           \
    return 0;                                                                                                   \
  } while (0)
  if (epi == EPI_SILU) XOT_MOE(EPI_SILU, false);
  if (out_f32) XOT_MOE(EPI_NONE, true);
  XOT_MOE(EPI_NONE, false);
#undef XOT_MOE
}

template <int EPI, bool F32>
static int stream8_dispatch(const uint16_t* X, int ldx, const uint8_t* W8p, const float* wscale, int K,
                            const uint16_t* bias, const uint16_t* R, int ldr, void* Y, int ldy, float* ws,
                            long ws_elems, int M, int N, int ntw, int S, bool reduce, hipStream_t st) {
  const uint16_t* W = reinterpret_cast<const uint16_t*>(W8p);
  if (EPI == EPI_SILU && ntw == 1) ntw = 2;
  if (ntw != 1 && ntw != 2 && ntw != 4) return -1;
  const int mt = (M + 15) / 16;
  if (ntw == 4 && mt <= 2) ntw = 2;
  if (N % (64 * ntw) != 0 || S < 1 || K % (S * 128) != 0) return -1;
  if (S > 1 && (ws == nullptr || ws_elems < (long)S * M * N)) return -1;
#define XOT_S8(MTV, KSV)                                                                                            \
  do {                                                                                                              \
    if (ntw == 1 && EPI != EPI_SILU)                                                                                \
      stream_launch<MTV, 1, KSV, EPI, F32, true, true>(X, ldx, W, K, bias, R, ldr, Y, ldy, ws, M, N, K, S, reduce,  \
                                                       st, wscale);                                          \
    else if (ntw == 4 && MTV >= 4)                                                                                  \
      stream_launch<MTV, 4, KSV, EPI, F32, true, true>(X, ldx, W, K, bias, R, ldr, Y, ldy, ws, M, N, K, S, reduce,  \
                                                       st, wscale);                                          \
    else                                                                                                            \
      stream_launch<MTV, 2, KSV, EPI, F32, true, true>(X, ldx, W, K, bias, R, ldr, Y, ldy, ws, M, N, K, S, reduce,  \
                                                       st, wscale);                                          \
    return 0;                                                                                                       \
  } while (0)
  // (256-deep k-chunks for small M -- the bf16 kernel's bytes in flight per chunk -- measured no faster)
  if (mt <= 1) XOT_S8(1, 4);
  if (mt <= 2) XOT_S8(2, 4);
  if (mt <= 4) XOT_S8(4, 4);
  XOT_S8(8, 4);  // M > 128: 128-row blocks (see stream_dispatch)
#undef XOT_S8
}

int launch_gemm_stream8(const uint16_t* X, int ldx, const uint8_t* W, const float* wscale, const uint16_t* bias,
                        const uint16_t* R, int ldr, void* Y, int ldy, bool out_f32, int epi, float* ws, long ws_elems,
                        int M, int N, int K, int ntw, int S, bool reduce, hipStream_t s) {
  if (M <= 0) return 0;
  if (epi == EPI_SILU)
    return out_f32 ? -1 : stream8_dispatch<EPI_SILU, false>(X, ldx, W, wscale, K, bias, R, ldr, Y, ldy, ws, ws_elems, M, N, ntw, S, reduce, s);
  if (epi == EPI_RESID)
    return out_f32 ? -1 : stream8_dispatch<EPI_RESID, false>(X, ldx, W, wscale, K, bias, R, ldr, Y, ldy, ws, ws_elems, M, N, ntw, S, reduce, s);
  return out_f32 ? stream8_dispatch<EPI_NONE, true>(X, ldx, W, wscale, K, bias, R, ldr, Y, ldy, ws, ws_elems, M, N, ntw, S, reduce, s)
                 : stream8_dispatch<EPI_NONE, false>(X, ldx, W, wscale, K, bias, R, ldr, Y, ldy, ws, ws_elems, M, N, ntw, S, reduce, s);
}

template <int NTW, int EPI, int PM>
static void stream_norm_launch(const uint16_t* W, const uint16_t* bias, void* Y, int ldy, float* ws, int N, int K,
                               int S, bool reduce, const NormPro& np, hipStream_t st) {
  const int kper = K / S;
  const dim3 grid(N / (64 * NTW), S);
  const size_t smem = (size_t)kper * 2;  // the normalised K slice (<= 16 KB at K = 8192)
  if (S == 1) {
    gemm_stream_kernel<1, NTW, 4, EPI, false, false, true, 2, 0, false, PM><<<grid, 256, smem, st>>>(
        nullptr, 0, W, K, bias, nullptr, 0, Y, ldy, nullptr, 1, N, kper, 1, nullptr, nullptr, nullptr, 0L, nullptr,
        0L, 0L, np);
    return;
  }
  gemm_stream_kernel<1, NTW, 4, EPI, false, true, true, 2, 0, false, PM><<<grid, 256, smem, st>>>(
      nullptr, 0, W, K, bias, nullptr, 0, Y, ldy, ws, 1, N, kper, 1, nullptr, nullptr, nullptr, 0L, nullptr, 0L, 0L,
      np);
  if (!reduce) return;
  const int ncol = EPI == EPI_SILU ? N / 2 : N;
  splitk_reduce_kernel<EPI, false><<<(ncol / 8 + 255) / 256, 256, 0, st>>>(ws, S, 1, N, bias, nullptr, 0, Y, ldy);
}

// o_proj of a batch-1 decode step with the attention's partition merge in its prologue: split-K slabs only (the
// consumer -- splitk_resid_rmsnorm or the next GEMM's norm prologue -- adds them to the residual)
int launch_gemm_stream_merge(const uint16_t* W, float* ws, long ws_elems, int N, int K, int ntw, int S,
                             const NormPro& np, hipStream_t s) {
  if (ntw == 4) ntw = 2;
  if (ntw != 1 && ntw != 2) return -1;
  if (S < 2 || N % (64 * ntw) != 0 || K % (S * 128) != 0 || (long)(K / S) * 2 > 65536) return -1;
  if (ws == nullptr || ws_elems < (long)S * N || np.mo == nullptr || np.ml == nullptr || np.ctx == nullptr ||
      np.nparts < 1 || np.ppp < 1 || np.dh <= 0 || np.dh % 4 != 0 || K % np.dh != 0)
    return -1;
  const int kper = K / S;
  const dim3 grid(N / (64 * ntw), S);
  const size_t smem = (size_t)kper * 2;
  if (ntw == 1)
    gemm_stream_kernel<1, 1, 4, EPI_NONE, false, true, true, 2, 0, false, 0, true><<<grid, 256, smem, s>>>(
        nullptr, 0, W, K, nullptr, nullptr, 0, nullptr, N, ws, 1, N, kper, 1, nullptr, nullptr, nullptr, 0L, nullptr,
        0L, 0L, np);
  else
    gemm_stream_kernel<1, 2, 4, EPI_NONE, false, true, true, 2, 0, false, 0, true><<<grid, 256, smem, s>>>(
        nullptr, 0, W, K, nullptr, nullptr, 0, nullptr, N, ws, 1, N, kper, 1, nullptr, nullptr, nullptr, 0L, nullptr,
        0L, 0L, np);
  return 0;
}

int launch_gemm_stream_norm(const uint16_t* W, const uint16_t* bias, void* Y, int ldy, int epi, float* ws,
                            long ws_elems, int N, int K, int ntw, int S, bool reduce, const NormPro& np,
                            hipStream_t s) {
  if (epi != EPI_NONE && epi != EPI_SILU) return -1;
  if (epi == EPI_SILU || ntw == 4) ntw = 2;  // one row: NTW 4 is never picked (stream_dispatch)
  if (ntw != 1 && ntw != 2) return -1;
  if (np.D != K || K % 8 != 0 || K > 8 * 256 * 4 || np.S < 0 || np.S > 8 || np.h == nullptr || np.lnw == nullptr || np.hout == nullptr)
    return -1;
  if (np.S > 0 && (np.ws == nullptr || np.sstride < K)) return -1;
  if (S < 1 || N % (64 * ntw) != 0 || K % (S * 128) != 0 || (long)(K / S) * 2 > 65536) return -1;
  if (S > 1 && (ws == nullptr || ws == np.ws || ws_elems < (long)S * N)) return -1;
  const int pm = (K / 8 + 255) / 256;  // 16-B chunks of the row per thread
  auto go = [&](auto pmc) {
    constexpr int PM = decltype(pmc)::value;
    if (epi == EPI_SILU)
      stream_norm_launch<2, EPI_SILU, PM>(W, bias, Y, ldy, ws, N, K, S, reduce, np, s);
    else if (ntw == 1)
      stream_norm_launch<1, EPI_NONE, PM>(W, bias, Y, ldy, ws, N, K, S, reduce, np, s);
    else
      stream_norm_launch<2, EPI_NONE, PM>(W, bias, Y, ldy, ws, N, K, S, reduce, np, s);
  };
  if (pm <= 1)
    go(std::integral_constant<int, 1>());
  else if (pm == 2)
    go(std::integral_constant<int, 2>());
  else
    go(std::integral_constant<int, 4>());
  return 0;
}

int launch_gemm_stream(const uint16_t* X, int ldx, const uint16_t* W, int ldw, const uint16_t* bias,
                       const uint16_t* R, int ldr, void* Y, int ldy, bool out_f32, int epi, float* ws, long ws_elems,
                       int M, int N, int K, int ntw, int S, bool wshuf, bool reduce,
                       hipStream_t s) {
  if (M <= 0) return 0;
  if (epi == EPI_SILU)
    return out_f32 ? stream_dispatch<EPI_SILU, true>(X, ldx, W, ldw, bias, R, ldr, Y, ldy, ws, ws_elems, M, N, K, ntw, S, wshuf, reduce, s)
                   : stream_dispatch<EPI_SILU, false>(X, ldx, W, ldw, bias, R, ldr, Y, ldy, ws, ws_elems, M, N, K, ntw, S, wshuf, reduce, s);
  if (epi == EPI_RESID)
    return out_f32 ? -1 : stream_dispatch<EPI_RESID, false>(X, ldx, W, ldw, bias, R, ldr, Y, ldy, ws, ws_elems, M, N, K, ntw, S, wshuf, reduce, s);
  return out_f32 ? stream_dispatch<EPI_NONE, true>(X, ldx, W, ldw, bias, R, ldr, Y, ldy, ws, ws_elems, M, N, K, ntw, S, wshuf, reduce, s)
                 : stream_dispatch<EPI_NONE, false>(X, ldx, W, ldw, bias, R, ldr, Y, ldy, ws, ws_elems, M, N, K, ntw, S, wshuf, reduce, s);
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

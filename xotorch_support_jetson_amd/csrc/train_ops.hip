// Training-path kernels: fused cross-entropy (forward + backward) and fused AdamW.
//
// The reference routes `xot train` through Node.enqueue_example -> engine.train(...) but never
// implements the engine side (xotorch/orchestration/node.py:210-345, inference_engine.py:34-35);
// these kernels are the loss/optimizer half of the train step this framework actually runs.
#include "common.h"
#include "kernels.h"

namespace xot {

template <typename T>
__device__ __forceinline__ float ldf(const T* p, long i);
template <>
__device__ __forceinline__ float ldf<float>(const float* p, long i) { return p[i]; }
template <>
__device__ __forceinline__ float ldf<uint16_t>(const uint16_t* p, long i) { return bf2f(p[i]); }

__device__ __forceinline__ void block_reduce_max_sum(float& m, float& s, float* sm, float* ss) {
  // combine (max, sum-of-exp relative to max) across the 256-thread block
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
    const float mn = fmaxf(m, m2);
    s = s * __expf(m - mn) + s2 * __expf(m2 - mn);
    m = mn;
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sm[w] = m;
    ss[w] = s;
  }
  __syncthreads();
  m = sm[0];
  s = ss[0];
  for (int i = 1; i < 4; ++i) {
    const float mn = fmaxf(m, sm[i]);
    s = s * __expf(m - mn) + ss[i] * __expf(sm[i] - mn);
    m = mn;
  }
}

// loss[t] = lse(x_t) - x_t[target_t]   (0 and lse=0 when target < 0: ignored position)
template <typename T>
__global__ __launch_bounds__(256) void ce_fwd_kernel(const T* __restrict__ x, long ld, int V,
                                                     const int32_t* __restrict__ tgt, float* __restrict__ loss,
                                                     float* __restrict__ lse) {
  __shared__ float sm[4], ss[4];
  const int t = blockIdx.x;
  const T* row = x + (size_t)t * ld;
  float m = -INFINITY, s = 0.f;
  for (int i = threadIdx.x; i < V; i += 256) {
    const float v = ldf(row, i);
    if (v > m) {
      s = s * __expf(m - v) + 1.f;
      m = v;
    } else {
      s += __expf(v - m);
    }
  }
  if (m == -INFINITY) s = 0.f;
  block_reduce_max_sum(m, s, sm, ss);
  if (threadIdx.x == 0) {
    const float l = m + __logf(s);
    const int y = tgt[t];
    lse[t] = l;
    loss[t] = (y >= 0 && y < V) ? l - ldf(row, y) : 0.f;
  }
}

// dx[t, i] = gscale[t] * (softmax_i - [i == target])   (zero row for ignored positions)
template <typename T>
__global__ __launch_bounds__(256) void ce_bwd_kernel(const T* __restrict__ x, long ld, int V,
                                                     const int32_t* __restrict__ tgt, const float* __restrict__ lse,
                                                     const float* __restrict__ gscale, uint16_t* __restrict__ dx,
                                                     long ldd) {
  const int t = blockIdx.x;
  const T* row = x + (size_t)t * ld;
  uint16_t* drow = dx + (size_t)t * ldd;
  const int y = tgt[t];
  const bool ign = y < 0 || y >= V;
  const float l = lse[t], gs = gscale[t];
  for (int i = threadIdx.x; i < V; i += 256) {
    const float p = __expf(ldf(row, i) - l);
    drow[i] = ign ? (uint16_t)0 : f2bf(gs * (p - (i == y ? 1.f : 0.f)));
  }
}

// fp32 logits with V % 8 == 0 and 16-byte rows (the fused LM head's chunks): 16-byte loads, one online-softmax
// update per 4 values (the scalar forms ran at 3.3 / 4.0 TB/s on the 128k-vocab chunks)
__global__ __launch_bounds__(256) void ce_fwd_vec_kernel(const float* __restrict__ x, long ld, int V,
                                                        const int32_t* __restrict__ tgt, float* __restrict__ loss,
                                                        float* __restrict__ lse) {
  __shared__ float sm[4], ss[4];
  const int t = blockIdx.x;
  const f32x4* row = reinterpret_cast<const f32x4*>(x + (size_t)t * ld);
  // finite start: a thread with no elements (V / 4 < 256) must not feed exp(-inf - -inf) = NaN into the combine
  float m = -1e30f, s = 0.f;
  for (int i = threadIdx.x; i < V / 4; i += 256) {
    const f32x4 v = row[i];
    const float m4 = fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3]));
    if (m4 > m) {
      s *= __expf(m - m4);
      m = m4;
    }
    s += __expf(v[0] - m) + __expf(v[1] - m) + __expf(v[2] - m) + __expf(v[3] - m);
  }
  block_reduce_max_sum(m, s, sm, ss);
  if (threadIdx.x == 0) {
    const float l = m + __logf(s);
    const int y = tgt[t];
    lse[t] = l;
    loss[t] = (y >= 0 && y < V) ? l - x[(size_t)t * ld + y] : 0.f;
  }
}

__global__ __launch_bounds__(256) void ce_bwd_vec_kernel(const float* __restrict__ x, long ld, int V,
                                                        const int32_t* __restrict__ tgt, const float* __restrict__ lse,
                                                        const float* __restrict__ gscale, uint16_t* __restrict__ dx,
                                                        long ldd) {
  const int t = blockIdx.x;
  const f32x4* row = reinterpret_cast<const f32x4*>(x + (size_t)t * ld);
  s16x8* drow = reinterpret_cast<s16x8*>(dx + (size_t)t * ldd);
  const int y = tgt[t];
  const bool ign = y < 0 || y >= V;
  const float l = lse[t], gs = ign ? 0.f : gscale[t];
  for (int i = threadIdx.x; i < V / 8; i += 256) {
    const f32x4 a = row[2 * i], b = row[2 * i + 1];
    s16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float v = e < 4 ? a[e] : b[e - 4];
      o[e] = (short)f2bf(gs * (__expf(v - l) - (8 * i + e == y ? 1.f : 0.f)));
    }
    drow[i] = o;
  }
}

void launch_ce_fwd(const void* x, bool x_f32, long ld, int T, int V, const int32_t* tgt, float* loss, float* lse,
                   hipStream_t s) {
  if (T <= 0) return;
  if (x_f32 && V % 8 == 0 && ld % 4 == 0 && ((uintptr_t)x & 15) == 0) {
    ce_fwd_vec_kernel<<<T, 256, 0, s>>>((const float*)x, ld, V, tgt, loss, lse);
    return;
  }
  if (x_f32)
    ce_fwd_kernel<float><<<T, 256, 0, s>>>((const float*)x, ld, V, tgt, loss, lse);
  else
    ce_fwd_kernel<uint16_t><<<T, 256, 0, s>>>((const uint16_t*)x, ld, V, tgt, loss, lse);
}

void launch_ce_bwd(const void* x, bool x_f32, long ld, int T, int V, const int32_t* tgt, const float* lse,
                   const float* gscale, uint16_t* dx, long ldd, hipStream_t s) {
  if (T <= 0) return;
  if (x_f32 && V % 8 == 0 && ld % 4 == 0 && ldd % 8 == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)dx & 15) == 0) {
    ce_bwd_vec_kernel<<<T, 256, 0, s>>>((const float*)x, ld, V, tgt, lse, gscale, dx, ldd);
    return;
  }
  if (x_f32)
    ce_bwd_kernel<float><<<T, 256, 0, s>>>((const float*)x, ld, V, tgt, lse, gscale, dx, ldd);
  else
    ce_bwd_kernel<uint16_t><<<T, 256, 0, s>>>((const uint16_t*)x, ld, V, tgt, lse, gscale, dx, ldd);
}

// ---------------------------------------------------------------- AdamW
// fp32 master weights + fp32 moments; grads in bf16 (model dtype) or fp32; writes the bf16 model copy.
template <typename G>
__global__ __launch_bounds__(256) void adamw_kernel(float* __restrict__ p, const G* __restrict__ gr,
                                                    float* __restrict__ m, float* __restrict__ v,
                                                    uint16_t* __restrict__ p_bf16, long n, float lr, float b1,
                                                    float b2, float eps, float wd, float bc1, float bc2,
                                                    float gscale) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const float g = ldf(gr, i) * gscale;
    const float mi = b1 * m[i] + (1.f - b1) * g;
    const float vi = b2 * v[i] + (1.f - b2) * g * g;
    m[i] = mi;
    v[i] = vi;
    float pi = p[i];
    pi -= lr * ((mi / bc1) / (sqrtf(vi / bc2) + eps) + wd * pi);
    p[i] = pi;
    if (p_bf16 != nullptr) p_bf16[i] = f2bf(pi);
  }
}

void launch_adamw(float* p, const void* g, bool g_f32, float* m, float* v, uint16_t* p_bf16, long n, float lr,
                  float b1, float b2, float eps, float wd, int step, float gscale, hipStream_t s) {
  if (n <= 0) return;
  const float bc1 = 1.f - powf(b1, (float)step), bc2 = 1.f - powf(b2, (float)step);
  long gsz = (n + 255) / 256;
  const int grid = (int)(gsz > 8192 ? 8192 : gsz);
  if (g_f32)
    adamw_kernel<float><<<grid, 256, 0, s>>>(p, (const float*)g, m, v, p_bf16, n, lr, b1, b2, eps, wd, bc1, bc2, gscale);
  else
    adamw_kernel<uint16_t><<<grid, 256, 0, s>>>(p, (const uint16_t*)g, m, v, p_bf16, n, lr, b1, b2, eps, wd, bc1, bc2,
                                                gscale);
}

// ---------------------------------------------------------------- AdamW fused with the operand-layout refresh
// One 2-D projection weight W [N, K] (N, K multiples of 128): the AdamW update of a 128 x 128 tile, then the
// tile's bf16 values written straight into both own-GEMM operand images -- ws = shuffle(W) and wts =
// shuffle(W^T) (csrc/layout.hip modes 0 / 1, ops/weights_layout.py shuffle_for_stream) -- from LDS, instead
// of writing the bf16 copy and re-reading it twice in two relayout kernels after the step (~2 x 2 B per
// parameter of HBM traffic, ~10 ms of the Llama-3-8B step).  In both images a 16-row group x 128-column block
// is one contiguous 2048-element run: position ((k % 128) / 8) * 16 + row % 16 holds the row's 8-element
// granule, so every global store is a full 16 B and consecutive threads store consecutive granules.
// pb (nullable): the plain bf16 copy, for weights something else still reads (a tied embedding).
constexpr int AT_LD = 128 + 8;  // padded LDS rows: a 16-lane group reading 16 rows of one granule hits 64 banks

template <typename G>
__global__ __launch_bounds__(256) void adamw_tiled_kernel(float* __restrict__ p, const G* __restrict__ gr,
                                                          float* __restrict__ m, float* __restrict__ v,
                                                          uint16_t* __restrict__ pb, uint16_t* __restrict__ ws,
                                                          uint16_t* __restrict__ wts, int N, int K, float lr,
                                                          float b1, float b2, float eps, float wd, float bc1,
                                                          float bc2, float gscale) {
  __shared__ __attribute__((aligned(16))) uint16_t tr[128 * AT_LD];  // tile [n][k]
  __shared__ __attribute__((aligned(16))) uint16_t tt[128 * AT_LD];  // tile [k][n]
  const int n0 = blockIdx.y * 128, k0 = blockIdx.x * 128;
#pragma unroll 2
  for (int it = 0; it < 8; ++it) {
    const int i = threadIdx.x + 256 * it, row = i >> 4, cg = i & 15;
    const long off = (long)(n0 + row) * K + k0 + cg * 8;
    float gv[8];
    if constexpr (sizeof(G) == 2) {
      const s16x8 g8 = ld16(reinterpret_cast<const uint16_t*>(gr) + off);
#pragma unroll
      for (int e = 0; e < 8; ++e) gv[e] = bf2f(g8[e]);
    } else {
      const f32x4 ga = *reinterpret_cast<const f32x4*>(gr + off), gb = *reinterpret_cast<const f32x4*>(gr + off + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        gv[e] = ga[e];
        gv[4 + e] = gb[e];
      }
    }
    f32x4 pv[2], mv[2], vv[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      pv[h] = *reinterpret_cast<const f32x4*>(p + off + 4 * h);
      mv[h] = *reinterpret_cast<const f32x4*>(m + off + 4 * h);
      vv[h] = *reinterpret_cast<const f32x4*>(v + off + 4 * h);
    }
    s16x8 bv;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int h = e >> 2, j = e & 3;
      const float g = gv[e] * gscale;
      const float mi = b1 * mv[h][j] + (1.f - b1) * g;
      const float vi = b2 * vv[h][j] + (1.f - b2) * g * g;
      mv[h][j] = mi;
      vv[h][j] = vi;
      float pi = pv[h][j];
      pi -= lr * ((mi / bc1) / (sqrtf(vi / bc2) + eps) + wd * pi);
      pv[h][j] = pi;
      bv[e] = (short)f2bf(pi);
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      *reinterpret_cast<f32x4*>(p + off + 4 * h) = pv[h];
      *reinterpret_cast<f32x4*>(m + off + 4 * h) = mv[h];
      *reinterpret_cast<f32x4*>(v + off + 4 * h) = vv[h];
    }
    if (pb != nullptr) st16(pb + off, bv);
    st16(tr + row * AT_LD + cg * 8, bv);
#pragma unroll
    for (int e = 0; e < 8; ++e) tt[(cg * 8 + e) * AT_LD + row] = (uint16_t)bv[e];
  }
  __syncthreads();
  // 8 groups of 16 rows x 256 granules in each image
#pragma unroll 4
  for (int it = 0; it < 8; ++it) {
    const int i = threadIdx.x + 256 * it, blk = i >> 8, pos = i & 255, q8 = pos >> 4, r = pos & 15;
    st16(ws + ((long)((n0 >> 4) + blk) * (K / 128) + (k0 >> 7)) * 2048 + pos * 8,
         ld16(tr + (blk * 16 + r) * AT_LD + q8 * 8));
    st16(wts + ((long)((k0 >> 4) + blk) * (N / 128) + (n0 >> 7)) * 2048 + pos * 8,
         ld16(tt + (blk * 16 + r) * AT_LD + q8 * 8));
  }
}

int launch_adamw_tiled(float* p, const void* g, bool g_f32, float* m, float* v, uint16_t* pb, uint16_t* ws,
                       uint16_t* wts, int N, int K, float lr, float b1, float b2, float eps, float wd, int step,
                       float gscale, hipStream_t s) {
  if (N % 128 || K % 128 || N <= 0 || K <= 0) return -1;
  const float bc1 = 1.f - powf(b1, (float)step), bc2 = 1.f - powf(b2, (float)step);
  const dim3 grid(K / 128, N / 128);
  if (g_f32)
    adamw_tiled_kernel<float><<<grid, 256, 0, s>>>(p, (const float*)g, m, v, pb, ws, wts, N, K, lr, b1, b2, eps, wd,
                                                   bc1, bc2, gscale);
  else
    adamw_tiled_kernel<uint16_t><<<grid, 256, 0, s>>>(p, (const uint16_t*)g, m, v, pb, ws, wts, N, K, lr, b1, b2,
                                                      eps, wd, bc1, bc2, gscale);
  return 0;
}

// ---------------------------------------------------------------- multi-tensor sum of squares
// Gradient-norm clipping over every parameter's gradient in two launches instead of one torch norm kernel per
// tensor (195 for Llama-3-8B, 8.5 ms/step at ~1.9 TB/s, profiles/r5/train/trainprof_step_r5h.txt): block
// (c, t) sums the squares of chunk c of tensor t of a batch into part[t * maxc + c] (0 for chunks past the
// tensor's end), one reduce kernel then sums all partials into out[0].
constexpr int SUMSQ_CHUNK = 256 * 8 * 64;  // elements per block: 64 16-byte loads per thread

template <typename T>
__device__ __forceinline__ float sumsq_chunk(const T* __restrict__ p, long lo, long hi) {
  float acc = 0.f;
  constexpr int V = 16 / sizeof(T);  // elements per 16-byte load
  const bool aligned = ((uintptr_t)(p + lo) & 15) == 0;
  if (aligned) {
    const long nv = (hi - lo) / V;
    for (long i = threadIdx.x; i < nv; i += 256) {
      if constexpr (sizeof(T) == 2) {
        const s16x8 x = ld16(reinterpret_cast<const uint16_t*>(p) + lo + i * V);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float f = bf2f(x[j]);
          acc += f * f;
        }
      } else {
        const f32x4 x = *reinterpret_cast<const f32x4*>(p + lo + i * V);
        acc += x[0] * x[0] + x[1] * x[1] + x[2] * x[2] + x[3] * x[3];
      }
    }
    lo += nv * V;
  }
  for (long i = lo + threadIdx.x; i < hi; i += 256) {
    const float f = ldf(p, i);
    acc += f * f;
  }
  return acc;
}

__global__ __launch_bounds__(256) void multi_sumsq_kernel(SumsqBatch b, float* __restrict__ part, int maxc) {
  const int t = blockIdx.y, c = blockIdx.x;
  const long lo = (long)c * SUMSQ_CHUNK, n = b.n[t];
  float acc = 0.f;
  if (lo < n) {
    const long hi = lo + SUMSQ_CHUNK < n ? lo + SUMSQ_CHUNK : n;
    acc = b.f32[t] ? sumsq_chunk((const float*)b.p[t], lo, hi) : sumsq_chunk((const uint16_t*)b.p[t], lo, hi);
  }
  __shared__ float red[4];
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) part[(long)t * maxc + c] = (red[0] + red[1]) + (red[2] + red[3]);
}

// sum of part[0 .. n) into out[blockIdx.x] by a grid-stride over gridDim.x blocks (two launches: gridDim.x
// partials, then one block over them -- one block over the ~10^6 per-chunk partials took 1.5 ms)
__global__ __launch_bounds__(256) void sum_reduce_kernel(const float* __restrict__ part, long n,
                                                         float* __restrict__ out) {
  float acc = 0.f;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) acc += part[i];
  __shared__ float red[4];
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

int multi_sumsq_chunk() { return SUMSQ_CHUNK; }
constexpr int SUMSQ_RED_BLOCKS = 512;  // first reduce level (its partials live in part's first slots' tail)

void launch_multi_sumsq(const SumsqBatch* batches, int nbatch, int maxc, float* part, float* out, hipStream_t s) {
  for (int i = 0; i < nbatch; ++i)
    multi_sumsq_kernel<<<dim3(maxc, batches[i].count), 256, 0, s>>>(batches[i], part + (long)i * SUMSQ_MAXT * maxc,
                                                                     maxc);
  const long n = (long)nbatch * SUMSQ_MAXT * maxc;
  float* lvl = part + n;  // SUMSQ_RED_BLOCKS floats after the per-chunk partials (multi_sumsq_scratch)
  sum_reduce_kernel<<<SUMSQ_RED_BLOCKS, 256, 0, s>>>(part, n, lvl);
  sum_reduce_kernel<<<1, 256, 0, s>>>(lvl, SUMSQ_RED_BLOCKS, out);
}

long multi_sumsq_scratch(int nbatch, int maxc) { return (long)nbatch * SUMSQ_MAXT * maxc + SUMSQ_RED_BLOCKS; }

}  // namespace xot

// Memory-bound row kernels: RMSNorm (+fused residual add), RMSNorm backward,
// token-embedding gather, SiLU*mul (fwd/bwd) and rotary embedding
// (fused with the paged KV-cache write for inference, plain/inverse for training).
//
// Reference parity: these replace the torchtune RMSNorm / RoPE / KVCache.update /
// nn.Embedding / FeedForward activation that the reference runs through stock
// torch ops (xotorch/inference/torch/models/general_mha.py:33-63,77-120,
// xotorch/inference/torch/models/llm_utils.py:399-435,513-522).
// All loads/stores are 16 B per lane (8 x bf16); reductions are wave64 shuffles.
#include "common.h"
#include <cstdlib>
#include "kernels.h"

namespace xot {

// ---------------------------------------------------------------- RMSNorm fwd
// out = rmsnorm(x [+ res]) * w ; if res != null, res_out = bf16(x + res)
template <int MAXC>
__global__ __launch_bounds__(256) void rmsnorm_kernel(const uint16_t* __restrict__ x,
                                                      const uint16_t* __restrict__ res,
                                                      const uint16_t* __restrict__ w,
                                                      uint16_t* __restrict__ out,
                                                      uint16_t* __restrict__ res_out, int D, float eps) {
  __shared__ float red[4];
  const int row = blockIdx.x, tid = threadIdx.x, nchunk = D >> 3;
  const size_t base = (size_t)row * D;
  float v[MAXC][8];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < MAXC; ++i) {
    const int c = tid + i * 256;
    if (c < nchunk) {
      s16x8 a = ld16(x + base + c * 8);
      if (res != nullptr) {
        s16x8 b = ld16(res + base + c * 8);
        s16x8 h;
#pragma unroll
        for (int j = 0; j < 8; ++j) h[j] = (short)f2bf(bf2f(a[j]) + bf2f(b[j]));
        st16(res_out + base + c * 8, h);
        a = h;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        v[i][j] = bf2f(a[j]);
        ss += v[i][j] * v[i][j];
      }
    }
  }
  ss = wave_sum(ss);
  if ((tid & 63) == 0) red[tid >> 6] = ss;
  __syncthreads();
  ss = red[0] + red[1] + red[2] + red[3];
  const float inv = rsqrtf(ss / (float)D + eps);
#pragma unroll
  for (int i = 0; i < MAXC; ++i) {
    const int c = tid + i * 256;
    if (c < nchunk) {
      s16x8 wv = ld16(w + c * 8), o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (short)f2bf(v[i][j] * inv * bf2f(wv[j]));
      st16(out + base + c * 8, o);
    }
  }
}

void launch_rmsnorm(const uint16_t* x, const uint16_t* res, const uint16_t* w, uint16_t* out,
                    uint16_t* res_out, int rows, int D, float eps, hipStream_t s) {
  if (rows <= 0) return;
  const int nchunk = D / 8;
  if (nchunk <= 256)
    rmsnorm_kernel<1><<<rows, 256, 0, s>>>(x, res, w, out, res_out, D, eps);
  else if (nchunk <= 512)
    rmsnorm_kernel<2><<<rows, 256, 0, s>>>(x, res, w, out, res_out, D, eps);
  else if (nchunk <= 1024)
    rmsnorm_kernel<4><<<rows, 256, 0, s>>>(x, res, w, out, res_out, D, eps);
  else
    rmsnorm_kernel<8><<<rows, 256, 0, s>>>(x, res, w, out, res_out, D, eps);
}

// ---------------------------------------------------------------- split-K reduce + residual + RMSNorm
// One workgroup per row: h = bf16(h + bias + sum_s ws[s][row]) (in place), out = rmsnorm(h) * w.  Replaces
// the split-K reduce kernel of a residual projection (o_proj / down_proj) and the RMSNorm that follows it.
// SS > 0: exactly SS slabs, loads unrolled and issued together (a runtime slab loop waits for each load
// in turn: one row at decode batch 1 took 6.9 us); SS = 0: any S.
// NTH threads per row: 1024 for wide rows (D = 8192 at decode batch 512: 512 workgroups of 256 threads left 8 waves
// per CU and each thread's four chunks x (h + S slabs) loads partly serialised; 16 waves per row keep one chunk each)
template <int MAXC, int SS, int NTH = 256>
__global__ __launch_bounds__(NTH) void splitk_resid_rmsnorm_kernel(const float* __restrict__ ws, int S,
                                                                   size_t sstride, const uint16_t* __restrict__ bias,
                                                                   uint16_t* __restrict__ h,
                                                                   const uint16_t* __restrict__ w,
                                                                   uint16_t* __restrict__ out, int D, float eps) {
  __shared__ float red[NTH / 64];
  const int row = blockIdx.x, tid = threadIdx.x, nchunk = D >> 3;
  const size_t base = (size_t)row * D;
  float v[MAXC][8];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < MAXC; ++i) {
    const int c = tid + i * NTH;
    if (c < nchunk) {
      const s16x8 a = ld16(h + base + c * 8);
      float acc[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = bf2f(a[j]);
      if (bias != nullptr) {
        const s16x8 bv = ld16(bias + c * 8);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += bf2f(bv[j]);
      }
      const float* sp = ws + base + c * 8;
      if constexpr (SS > 0) {
        f32x4 p[SS][2];
#pragma unroll
        for (int sl = 0; sl < SS; ++sl) {
          p[sl][0] = *reinterpret_cast<const f32x4*>(sp + sl * sstride);
          p[sl][1] = *reinterpret_cast<const f32x4*>(sp + sl * sstride + 4);
        }
#pragma unroll
        for (int sl = 0; sl < SS; ++sl)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            acc[j] += p[sl][0][j];
            acc[4 + j] += p[sl][1][j];
          }
      } else {
        for (int sl = 0; sl < S; ++sl, sp += sstride) {
          const f32x4 p0 = *reinterpret_cast<const f32x4*>(sp), p1 = *reinterpret_cast<const f32x4*>(sp + 4);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            acc[j] += p0[j];
            acc[4 + j] += p1[j];
          }
        }
      }
      s16x8 hv;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        hv[j] = (short)f2bf(acc[j]);
        v[i][j] = bf2f(hv[j]);  // normalise the stored (bf16) stream, as the unfused path does
        ss += v[i][j] * v[i][j];
      }
      st16(h + base + c * 8, hv);
    }
  }
  ss = wave_sum(ss);
  if ((tid & 63) == 0) red[tid >> 6] = ss;
  __syncthreads();
  ss = 0.f;
#pragma unroll
  for (int k = 0; k < NTH / 64; ++k) ss += red[k];
  const float inv = rsqrtf(ss / (float)D + eps);
#pragma unroll
  for (int i = 0; i < MAXC; ++i) {
    const int c = tid + i * NTH;
    if (c < nchunk) {
      s16x8 wv = ld16(w + c * 8), o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (short)f2bf(v[i][j] * inv * bf2f(wv[j]));
      st16(out + base + c * 8, o);
    }
  }
}

void launch_splitk_resid_rmsnorm(const float* ws, int S, const uint16_t* bias, uint16_t* h, const uint16_t* w,
                                 uint16_t* out, int rows, int D, float eps, hipStream_t s) {
  if (rows <= 0) return;
  const int nchunk = D / 8;
  const size_t ss = (size_t)rows * D;
  auto go = [&](auto maxc, auto nth) {
    constexpr int MC = decltype(maxc)::value, NT = decltype(nth)::value;
#define XOT_SRR(SV) splitk_resid_rmsnorm_kernel<MC, SV, NT><<<rows, NT, 0, s>>>(ws, S, ss, bias, h, w, out, D, eps)
    switch (S) {
      case 1: XOT_SRR(1); break;
      case 2: XOT_SRR(2); break;
      case 3: XOT_SRR(3); break;
      case 4: XOT_SRR(4); break;
      case 6: XOT_SRR(6); break;
      case 8: XOT_SRR(8); break;
      default: XOT_SRR(0); break;
    }
#undef XOT_SRR
  };
  using I256 = std::integral_constant<int, 256>;
  if (nchunk <= 256)
    go(std::integral_constant<int, 1>(), I256());
  else if (nchunk <= 512)
    go(std::integral_constant<int, 2>(), I256());
  else if (nchunk <= 1024 && rows >= 256)  // 1024 threads per row: 16.4 -> 14.4 us at 512 x 8192 (r4 srr_wide)
    go(std::integral_constant<int, 1>(), std::integral_constant<int, 1024>());
  else if (nchunk <= 1024)
    go(std::integral_constant<int, 4>(), I256());
  else
    go(std::integral_constant<int, 8>(), I256());
}

// ---------------------------------------------------------------- RMSNorm bwd
// y = x * inv * w  (inv = rsqrt(mean(x^2)+eps))
// dx = inv * (w*dy - xhat * mean(xhat * w * dy)) (+ res: the residual stream's gradient joining here, so the
// training step needs no separate add kernel per residual join),  dw += sum_rows dy * xhat
// ROWS rows per block so the dw partial sum is flushed once per block.
constexpr int RMS_BWD_ROWS = 4;  // 512 workgroups at 2048 rows: the rows of a block run one after another
template <int MAXC>
__global__ __launch_bounds__(256) void rmsnorm_bwd_kernel(const uint16_t* __restrict__ x,
                                                          const uint16_t* __restrict__ w,
                                                          const uint16_t* __restrict__ dy,
                                                          uint16_t* __restrict__ dx, float* __restrict__ dw,
                                                          float* __restrict__ dw_part, int rows, int D, float eps,
                                                          const uint16_t* __restrict__ res) {
  __shared__ float red[2][4];
  const int tid = threadIdx.x, nchunk = D >> 3;
  float dwacc[MAXC][8];
#pragma unroll
  for (int i = 0; i < MAXC; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) dwacc[i][j] = 0.f;
  const int r0 = blockIdx.x * RMS_BWD_ROWS;
  for (int rr = 0; rr < RMS_BWD_ROWS; ++rr) {
    const int row = r0 + rr;
    if (row >= rows) break;
    const size_t base = (size_t)row * D;
    float xv[MAXC][8], gv[MAXC][8];
    float ss = 0.f, dot = 0.f;
#pragma unroll
    for (int i = 0; i < MAXC; ++i) {
      const int c = tid + i * 256;
      if (c < nchunk) {
        s16x8 a = ld16(x + base + c * 8), g = ld16(dy + base + c * 8), wv = ld16(w + c * 8);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          xv[i][j] = bf2f(a[j]);
          gv[i][j] = bf2f(g[j]);
          ss += xv[i][j] * xv[i][j];
          dot += xv[i][j] * gv[i][j] * bf2f(wv[j]);
        }
      }
    }
    ss = wave_sum(ss);
    dot = wave_sum(dot);
    if ((tid & 63) == 0) {
      red[0][tid >> 6] = ss;
      red[1][tid >> 6] = dot;
    }
    __syncthreads();
    ss = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    dot = red[1][0] + red[1][1] + red[1][2] + red[1][3];
    __syncthreads();
    const float inv = rsqrtf(ss / (float)D + eps);
    const float coef = dot * inv * inv / (float)D;  // mean(xhat*w*dy) * (1/inv) ... folded below
#pragma unroll
    for (int i = 0; i < MAXC; ++i) {
      const int c = tid + i * 256;
      if (c < nchunk) {
        s16x8 wv = ld16(w + c * 8), o, rv = {};
        if (res != nullptr) rv = ld16(res + base + c * 8);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float xhat = xv[i][j] * inv;
          o[j] = (short)f2bf(inv * (bf2f(wv[j]) * gv[i][j] - xv[i][j] * coef) + bf2f(rv[j]));
          dwacc[i][j] += gv[i][j] * xhat;
        }
        st16(dx + base + c * 8, o);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < MAXC; ++i) {
    const int c = tid + i * 256;
    if (c < nchunk) {
      if (dw_part != nullptr) {  // this block's partial row of dw; summed by rmsnorm_dw_reduce_kernel
        float* o = dw_part + (size_t)blockIdx.x * D + c * 8;
        *reinterpret_cast<f32x4*>(o) = f32x4{dwacc[i][0], dwacc[i][1], dwacc[i][2], dwacc[i][3]};
        *reinterpret_cast<f32x4*>(o + 4) = f32x4{dwacc[i][4], dwacc[i][5], dwacc[i][6], dwacc[i][7]};
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) atomicAdd(dw + c * 8 + j, dwacc[i][j]);
      }
    }
  }
}

// dw[c] += sum over the blocks' partial rows: grid (D / 256, RED_SPLIT), each block sums a slice of the
// partial rows (consecutive threads, consecutive columns) and adds it with one atomic per column
constexpr int RED_SPLIT = 32;
__global__ __launch_bounds__(256) void rmsnorm_dw_reduce_kernel(const float* __restrict__ part, int nblk, int D,
                                                                float* __restrict__ dw) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= D) return;
  const int per = (nblk + RED_SPLIT - 1) / RED_SPLIT, b0 = blockIdx.y * per, b1 = min(nblk, b0 + per);
  if (b0 >= b1) return;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  int b = b0;
  for (; b + 4 <= b1; b += 4) {
    a0 += part[(size_t)b * D + c];
    a1 += part[(size_t)(b + 1) * D + c];
    a2 += part[(size_t)(b + 2) * D + c];
    a3 += part[(size_t)(b + 3) * D + c];
  }
  for (; b < b1; ++b) a0 += part[(size_t)b * D + c];
  atomicAdd(dw + c, (a0 + a1) + (a2 + a3));
}

// dw_part (nullable, >= ceil(rows / RMS_BWD_ROWS) * D floats): per-block partials + one reduce kernel
// instead of every block's atomics on the same D words (512 blocks contending on 4096 addresses ran
// the training step's RMSNorm backward 1.9x slower than the atomic-free form).
void launch_rmsnorm_bwd(const uint16_t* x, const uint16_t* w, const uint16_t* dy, uint16_t* dx, float* dw,
                        float* dw_part, int rows, int D, float eps, hipStream_t s, const uint16_t* res) {
  if (rows <= 0) return;
  const int nchunk = D / 8;
  const int nblk = (rows + RMS_BWD_ROWS - 1) / RMS_BWD_ROWS;
  dim3 grid(nblk);
  if (nchunk <= 256)
    rmsnorm_bwd_kernel<1><<<grid, 256, 0, s>>>(x, w, dy, dx, dw, dw_part, rows, D, eps, res);
  else if (nchunk <= 512)
    rmsnorm_bwd_kernel<2><<<grid, 256, 0, s>>>(x, w, dy, dx, dw, dw_part, rows, D, eps, res);
  else if (nchunk <= 1024)
    rmsnorm_bwd_kernel<4><<<grid, 256, 0, s>>>(x, w, dy, dx, dw, dw_part, rows, D, eps, res);
  else
    rmsnorm_bwd_kernel<8><<<grid, 256, 0, s>>>(x, w, dy, dx, dw, dw_part, rows, D, eps, res);
  if (dw_part != nullptr)
    rmsnorm_dw_reduce_kernel<<<dim3((D + 255) / 256, RED_SPLIT), 256, 0, s>>>(dw_part, nblk, D, dw);
}

int rmsnorm_bwd_part_rows() { return RMS_BWD_ROWS; }

// ---------------------------------------------------------------- embedding
__global__ __launch_bounds__(256) void embedding_kernel(const int32_t* __restrict__ ids,
                                                        const uint16_t* __restrict__ table,
                                                        uint16_t* __restrict__ out, int D, int vocab) {
  const int t = blockIdx.x;
  int id = ids[t];
  id = id < 0 ? 0 : (id >= vocab ? vocab - 1 : id);  // never read out of bounds
  const uint16_t* src = table + (size_t)id * D;
  uint16_t* dst = out + (size_t)t * D;
  for (int c = threadIdx.x; c < (D >> 3); c += 256) st16(dst + c * 8, ld16(src + c * 8));
}

void launch_embedding(const int32_t* ids, const uint16_t* table, uint16_t* out, int T, int D, int vocab,
                      hipStream_t s) {
  if (T <= 0) return;
  embedding_kernel<<<T, 256, 0, s>>>(ids, table, out, D, vocab);
}

// ---------------------------------------------------------------- SiLU * mul
// gu: [T, 2F] = [gate | up]; out [T, F] = silu(gate) * up
__global__ __launch_bounds__(256) void silu_mul_kernel(const uint16_t* __restrict__ gu, uint16_t* __restrict__ out,
                                                       int F, long total_chunks) {
  const int fc = F >> 3;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total_chunks; i += (long)gridDim.x * 256) {
    const long t = i / fc, c = i % fc;
    s16x8 g = ld16(gu + t * 2 * F + c * 8), u = ld16(gu + t * 2 * F + F + c * 8), o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (short)f2bf(silu(bf2f(g[j])) * bf2f(u[j]));
    st16(out + t * F + c * 8, o);
  }
}

// dgu[:, :F] = dout * up * dsilu(g),  dgu[:, F:] = dout * silu(g)
__global__ __launch_bounds__(256) void silu_mul_bwd_kernel(const uint16_t* __restrict__ gu,
                                                           const uint16_t* __restrict__ dout,
                                                           uint16_t* __restrict__ dgu, int F, long total_chunks) {
  const int fc = F >> 3;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total_chunks; i += (long)gridDim.x * 256) {
    const long t = i / fc, c = i % fc;
    s16x8 g = ld16(gu + t * 2 * F + c * 8), u = ld16(gu + t * 2 * F + F + c * 8), d = ld16(dout + t * F + c * 8);
    s16x8 dg, du;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float gf = bf2f(g[j]), uf = bf2f(u[j]), df = bf2f(d[j]);
      const float sg = 1.0f / (1.0f + __expf(-gf));
      const float s = gf * sg;
      dg[j] = (short)f2bf(df * uf * (sg * (1.0f + gf * (1.0f - sg))));
      du[j] = (short)f2bf(df * s);
    }
    st16(dgu + t * 2 * F + c * 8, dg);
    st16(dgu + t * 2 * F + F + c * 8, du);
  }
}

// gu: [T, 2F] with gate/up interleaved in 16-column tiles (the fused gate_up weight layout):
// cols [32j, 32j+16) = gate_{16j..16j+15}, [32j+16, 32j+32) = up_{16j..}; out [T, F]
__global__ __launch_bounds__(256) void silu_mul_il_kernel(const uint16_t* __restrict__ gu, uint16_t* __restrict__ out,
                                                          int F, long total_chunks) {
  const int fc = F >> 3;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total_chunks; i += (long)gridDim.x * 256) {
    const long t = i / fc;
    const int o = (int)(i % fc) * 8, j = o >> 4, w = o & 15;
    const uint16_t* row = gu + t * 2 * F;
    s16x8 g = ld16(row + 32 * j + w), u = ld16(row + 32 * j + 16 + w), r;
#pragma unroll
    for (int k = 0; k < 8; ++k) r[k] = (short)f2bf(silu(bf2f(g[k])) * bf2f(u[k]));
    st16(out + t * F + o, r);
  }
}

static int grid_for(long chunks) {
  long g = (chunks + 255) / 256;
  return (int)(g < 4096 ? (g < 1 ? 1 : g) : 4096);
}

void launch_silu_mul(const uint16_t* gu, uint16_t* out, int T, int F, hipStream_t s) {
  const long chunks = (long)T * (F / 8);
  if (chunks <= 0) return;
  silu_mul_kernel<<<grid_for(chunks), 256, 0, s>>>(gu, out, F, chunks);
}
void launch_silu_mul_il(const uint16_t* gu, uint16_t* out, int T, int F, hipStream_t s) {
  const long chunks = (long)T * (F / 8);
  if (chunks <= 0) return;
  silu_mul_il_kernel<<<grid_for(chunks), 256, 0, s>>>(gu, out, F, chunks);
}
void launch_silu_mul_bwd(const uint16_t* gu, const uint16_t* dout, uint16_t* dgu, int T, int F, hipStream_t s) {
  const long chunks = (long)T * (F / 8);
  if (chunks <= 0) return;
  silu_mul_bwd_kernel<<<grid_for(chunks), 256, 0, s>>>(gu, dout, dgu, F, chunks);
}

// ---------------------------------------------------------------- RoPE
// HF rotate-half convention (no torchtune q/k permute needed, cf. llm_utils.py:126-134):
//   o[i]      = x[i] * cos[i] - x[i+h] * sin[i]
//   o[i+h]    = x[i+h] * cos[i] + x[i] * sin[i]        (h = Dh/2)
// cos_sin: [max_pos, Dh] fp32, row p = [cos(p*f_0..f_{h-1}) | sin(...)]
__device__ __forceinline__ void rope4(const uint16_t* __restrict__ src, uint16_t* __restrict__ dst,
                                      const float* __restrict__ cs, int i, int half, float sgn) {
  const s16x4 a = *reinterpret_cast<const s16x4*>(src + i);
  const s16x4 b = *reinterpret_cast<const s16x4*>(src + i + half);
  const f32x4 c = *reinterpret_cast<const f32x4*>(cs + i);
  const f32x4 sn = *reinterpret_cast<const f32x4*>(cs + half + i);
  s16x4 oa, ob;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float x0 = bf2f(a[j]), x1 = bf2f(b[j]), sj = sgn * sn[j];
    oa[j] = (short)f2bf(x0 * c[j] - x1 * sj);
    ob[j] = (short)f2bf(x1 * c[j] + x0 * sj);
  }
  *reinterpret_cast<s16x4*>(dst + i) = oa;
  *reinterpret_cast<s16x4*>(dst + i + half) = ob;
}

// qkv [T, (H + 2*Hkv) * Dh]  ->  q_out [T, H, Dh] (rotated), k -> k_cache (rotated), v -> v_cache
// k_cache: [num_blocks, Hkv, BS, Dh]   v_cache: [num_blocks, Hkv, BS / 8, Dh, 8]  (V chunk-major per page,
// common.h v_page_off, so the P.V MFMA operand is contiguous along keys)
__global__ __launch_bounds__(256) void rope_kv_write_kernel(const uint16_t* __restrict__ qkv,
                                                            const int32_t* __restrict__ pos,
                                                            const float* __restrict__ cos_sin,
                                                            const int64_t* __restrict__ slots,
                                                            uint16_t* __restrict__ q_out, uint16_t* __restrict__ kc,
                                                            uint16_t* __restrict__ vc, int H, int Hkv, int Dh, int BS,
                                                            int max_pos, long nslots, int skip_v) {
  const int t = blockIdx.x;
  const int half = Dh >> 1, qpr = half >> 2;  // 4-wide pair-groups per head
  int p = pos[t];
  p = p < 0 ? 0 : (p >= max_pos ? max_pos - 1 : p);
  const float* cs = cos_sin + (size_t)p * Dh;
  const uint16_t* row = qkv + (size_t)t * (H + 2 * Hkv) * Dh;
  const int64_t slot = slots[t] < nslots ? slots[t] : -1;  // out-of-range slot: skip the write
  const long blk = slot >= 0 ? slot / BS : 0;
  const int off = slot >= 0 ? (int)(slot % BS) : 0;
  const int nrot = (H + Hkv) * qpr;
  for (int w = threadIdx.x; w < nrot; w += 256) {
    const int h = w / qpr, i = (w % qpr) * 4;
    if (h < H) {
      rope4(row + h * Dh, q_out + ((size_t)t * H + h) * Dh, cs, i, half, 1.f);
    } else if (slot >= 0) {
      const int kh = h - H;
      uint16_t* dst = kc + (((size_t)blk * Hkv + kh) * BS + off) * Dh;
      rope4(row + h * Dh, dst, cs, i, half, 1.f);
    }
  }
  if (slot < 0 || skip_v) return;
  const int nv = Hkv * Dh;
  const uint16_t* vsrc = row + (H + Hkv) * Dh;
  for (int w = threadIdx.x; w < nv; w += 256) {
    const int kh = w / Dh, d = w % Dh;
    vc[((size_t)blk * Hkv + kh) * Dh * BS + v_page_off(off, d, Dh)] = vsrc[w];
  }
}

// Same, straight from the split-K fp32 slabs of the QKV projection (ws [S][T][N], N = (H + 2*Hkv)*Dh):
// sum the slabs (+ bias), round to bf16 exactly as the separate reduce would, rotate, write -- one
// pass instead of reduce (write bf16 qkv) + rope (read it back), and one launch less per layer.
// Grid (T, item blocks): one thread per work item (a rotated 4+4 pair of q / k, or 4 values of v), the
// slab loads of an item issued together (SS > 0: exactly SS slabs), so a decode step of one token is
// a single round trip, not S dependent ones.
template <int SS>
__device__ __forceinline__ f32x4 slab_sum4(const float* __restrict__ ws, int S, size_t sstride,
                                           const uint16_t* __restrict__ bias, int col) {
  f32x4 a;
  if constexpr (SS > 0) {
    f32x4 p[SS];
#pragma unroll
    for (int k = 0; k < SS; ++k) p[k] = *reinterpret_cast<const f32x4*>(ws + k * sstride + col);
    a = p[0];
#pragma unroll
    for (int k = 1; k < SS; ++k) a += p[k];
  } else {
    a = *reinterpret_cast<const f32x4*>(ws + col);
    for (int k = 1; k < S; ++k) a += *reinterpret_cast<const f32x4*>(ws + k * sstride + col);
  }
  if (bias != nullptr) {
    const s16x4 b = *reinterpret_cast<const s16x4*>(bias + col);
#pragma unroll
    for (int j = 0; j < 4; ++j) a[j] += bf2f(b[j]);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) a[j] = bf2f(f2bf(a[j]));
  return a;
}

template <int SS>
__global__ __launch_bounds__(256) void splitk_rope_kv_write_kernel(
    const float* __restrict__ ws, int S, long sstride, const uint16_t* __restrict__ bias,
    const int32_t* __restrict__ pos, const float* __restrict__ cos_sin, const int64_t* __restrict__ slots,
    uint16_t* __restrict__ q_out, uint16_t* __restrict__ kc, uint16_t* __restrict__ vc, int H, int Hkv, int Dh, int BS,
    int max_pos, long nslots) {
  const int t = blockIdx.x;
  const int w = blockIdx.y * 256 + threadIdx.x;
  const int half = Dh >> 1, qpr = half >> 2;
  const int N = (H + 2 * Hkv) * Dh;
  const int nrot = (H + Hkv) * qpr, nv4 = Hkv * Dh / 4;
  if (w >= nrot + nv4) return;
  const float* row = ws + (size_t)t * N;
  const int64_t slot = slots[t] < nslots ? slots[t] : -1;
  const long blk = slot >= 0 ? slot / BS : 0;
  const int off = slot >= 0 ? (int)(slot % BS) : 0;
  if (w < nrot) {
    const int h = w / qpr, i = (w % qpr) * 4;
    uint16_t* dst;
    if (h < H) {
      dst = q_out + ((size_t)t * H + h) * Dh;
    } else if (slot >= 0) {
      dst = kc + (((size_t)blk * Hkv + (h - H)) * BS + off) * Dh;
    } else {
      return;
    }
    int p = pos[t];
    p = p < 0 ? 0 : (p >= max_pos ? max_pos - 1 : p);
    const float* cs = cos_sin + (size_t)p * Dh;
    const f32x4 a = slab_sum4<SS>(row, S, sstride, bias, h * Dh + i);
    const f32x4 b = slab_sum4<SS>(row, S, sstride, bias, h * Dh + i + half);
    const f32x4 c = *reinterpret_cast<const f32x4*>(cs + i);
    const f32x4 sn = *reinterpret_cast<const f32x4*>(cs + half + i);
    s16x4 oa, ob;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      oa[j] = (short)f2bf(a[j] * c[j] - b[j] * sn[j]);
      ob[j] = (short)f2bf(b[j] * c[j] + a[j] * sn[j]);
    }
    *reinterpret_cast<s16x4*>(dst + i) = oa;
    *reinterpret_cast<s16x4*>(dst + i + half) = ob;
    return;
  }
  if (slot < 0) return;
  const int e = 4 * (w - nrot), kh = e / Dh, d = e % Dh;
  const f32x4 v = slab_sum4<SS>(row, S, sstride, bias, (H + Hkv) * Dh + e);
  uint16_t* dst = vc + ((size_t)blk * Hkv + kh) * Dh * BS + v_page_off(off, d, Dh);
#pragma unroll
  for (int j = 0; j < 4; ++j) dst[8 * j] = f2bf(v[j]);  // dims d .. d+3: 16 B apart in one 64-B span
}

void launch_splitk_rope_kv_write(const float* ws, int S, const uint16_t* bias, const int32_t* pos,
                                 const float* cos_sin, const int64_t* slots, uint16_t* q_out, uint16_t* kc,
                                 uint16_t* vc, int T, int H, int Hkv, int Dh, int BS, int max_pos, long nslots,
                                 hipStream_t s) {
  if (T <= 0) return;
  const long sstride = (long)T * (H + 2 * Hkv) * Dh;
  const int items = (H + Hkv) * (Dh / 8) + Hkv * Dh / 4;
  const dim3 grid(T, (items + 255) / 256);
#define XOT_SRK(SV)                                                                                            \
  splitk_rope_kv_write_kernel<SV><<<grid, 256, 0, s>>>(ws, S, sstride, bias, pos, cos_sin, slots, q_out, kc, vc, H, \
                                                       Hkv, Dh, BS, max_pos, nslots)
  switch (S) {
    case 1: XOT_SRK(1); break;
    case 2: XOT_SRK(2); break;
    case 3: XOT_SRK(3); break;
    case 4: XOT_SRK(4); break;
    case 6: XOT_SRK(6); break;
    case 8: XOT_SRK(8); break;
    default: XOT_SRK(0); break;
  }
#undef XOT_SRK
}

// V of prefill-sized T: the per-token kernel above writes a token's V as Hkv * Dh scattered 2-byte stores.  Here a
// workgroup takes 64 consecutive tokens of one KV head through LDS: each group of 8 tokens whose slots are one
// aligned 8-key chunk of a page (every group of a prefill chunk that starts on a page boundary) leaves as Dh
// 16-B stores of [8 keys] runs, a wave's 64 dims 1 KB contiguous; other groups fall back to per-token stores.
constexpr int RKV_TOK = 64;
__global__ __launch_bounds__(256) void v_write_tiled_kernel(const uint16_t* __restrict__ qkv,
                                                            const int64_t* __restrict__ slots,
                                                            uint16_t* __restrict__ vc, int T, int H, int Hkv, int Dh,
                                                            int BS, long nslots) {
  extern __shared__ uint16_t vt[];  // [RKV_TOK][Dh + 2]
  __shared__ long cslot[RKV_TOK / 8];  // first slot of each 8-token group when it is one aligned chunk, else -1
  const int t0 = blockIdx.x * RKV_TOK, nt = min(RKV_TOK, T - t0), kh = blockIdx.y;
  const int rowlen = (H + 2 * Hkv) * Dh, VLD = Dh + 2, cpr = Dh / 8;
  for (int w = threadIdx.x; w < nt * cpr; w += 256) {
    const int tt = w / cpr, cc = w % cpr;
    const s16x8 v = ld16(qkv + (size_t)(t0 + tt) * rowlen + (H + Hkv + kh) * Dh + cc * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) vt[tt * VLD + cc * 8 + j] = (uint16_t)v[j];
  }
  if (threadIdx.x < RKV_TOK / 8) {
    const int tt0 = threadIdx.x * 8;
    long s0 = tt0 + 8 <= nt ? (long)slots[t0 + tt0] : -1;
    if (s0 < 0 || s0 % 8 != 0 || s0 + 8 > nslots) s0 = -1;
    for (int i = 1; i < 8 && s0 >= 0; ++i)
      if ((long)slots[t0 + tt0 + i] != s0 + i) s0 = -1;
    cslot[threadIdx.x] = s0;
  }
  __syncthreads();
  const size_t head = (size_t)kh * Dh * BS;
  for (int w = threadIdx.x; w < ((nt + 7) / 8) * Dh; w += 256) {
    const int cg = w / Dh, d = w % Dh, tt0 = cg * 8;
    const long s0 = cslot[cg];
    if (s0 >= 0) {
      s16x8 v;
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = (short)vt[(tt0 + i) * VLD + d];
      st16(vc + (size_t)(s0 / BS) * Hkv * Dh * BS + head + v_page_off((int)(s0 % BS), d, Dh), v);
    } else {
      for (int i = 0; i < 8 && tt0 + i < nt; ++i) {
        const int64_t slot = slots[t0 + tt0 + i] < nslots ? slots[t0 + tt0 + i] : -1;
        if (slot >= 0)
          vc[(size_t)(slot / BS) * Hkv * Dh * BS + head + v_page_off((int)(slot % BS), d, Dh)] = vt[(tt0 + i) * VLD + d];
      }
    }
  }
}

void launch_rope_kv_write(const uint16_t* qkv, const int32_t* pos, const float* cos_sin, const int64_t* slots,
                          uint16_t* q_out, uint16_t* kc, uint16_t* vc, int T, int H, int Hkv, int Dh, int BS,
                          int max_pos, long nslots, hipStream_t s) {
  if (T <= 0) return;
  const bool vt = T >= 4 * RKV_TOK && Dh % 8 == 0;  // V through LDS tiles (prefill chunks)
  rope_kv_write_kernel<<<T, 256, 0, s>>>(qkv, pos, cos_sin, slots, q_out, kc, vc, H, Hkv, Dh, BS, max_pos, nslots,
                                         vt ? 1 : 0);
  if (vt)
    v_write_tiled_kernel<<<dim3((T + RKV_TOK - 1) / RKV_TOK, Hkv), 256, (size_t)RKV_TOK * (Dh + 2) * 2, s>>>(
        qkv, slots, vc, T, H, Hkv, Dh, BS, nslots);
}

// plain rotation of x [T, nh, Dh] (row stride ld elements between tokens) -> y (may alias x);
// inverse=1 applies the transpose rotation (the backward of the forward rotation)
__global__ __launch_bounds__(256) void rope_apply_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ y,
                                                         const int32_t* __restrict__ pos,
                                                         const float* __restrict__ cos_sin, int nh, int Dh,
                                                         long ldx, long ldy, int max_pos, float sgn) {
  const int t = blockIdx.x;
  const int half = Dh >> 1, qpr = half >> 2;
  int p = pos[t];
  p = p < 0 ? 0 : (p >= max_pos ? max_pos - 1 : p);
  const float* cs = cos_sin + (size_t)p * Dh;
  for (int w = threadIdx.x; w < nh * qpr; w += 256) {
    const int h = w / qpr, i = (w % qpr) * 4;
    rope4(x + t * ldx + h * Dh, y + t * ldy + h * Dh, cs, i, half, sgn);
  }
}

void launch_rope_apply(const uint16_t* x, uint16_t* y, const int32_t* pos, const float* cos_sin, int T, int nh,
                       int Dh, long ldx, long ldy, int max_pos, bool inverse, hipStream_t s) {
  if (T <= 0) return;
  rope_apply_kernel<<<T, 256, 0, s>>>(x, y, pos, cos_sin, nh, Dh, ldx, ldy, max_pos, inverse ? -1.f : 1.f);
}

}  // namespace xot

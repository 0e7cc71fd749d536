// Mixture-of-experts routing and combine for gfx950 (Mixtral-style top-k softmax gating).
//
// moe_route: one workgroup of 1024 threads.  Per token: softmax over the E router logits, top-k,
// renormalised weights; per expert a count (LDS atomics), an exclusive scan to slot offsets, and each
// (token, j) gets a slot in the expert-sorted order.  Slot order inside an expert is arbitrary: the
// grouped GEMM treats rows independently and the combine sums each token's k slots in j order, so
// results do not depend on it.  Everything stays on the device (graph-capturable).
// moe_combine: h[t] += sum_j w[t, j] * y[slot_of[t, j]] with the expert outputs y in fp32.
#include "common.h"
#include "kernels.h"

namespace xot {

constexpr int MOE_MAX_E = 64;
constexpr int MOE_MAX_K = 8;

__global__ __launch_bounds__(1024) void moe_route_kernel(const float* __restrict__ logits, int T, int E, int k,
                                                         float* __restrict__ topw, int32_t* __restrict__ topi,
                                                         int32_t* __restrict__ slot_of,
                                                         int32_t* __restrict__ sorted_tok, int32_t* __restrict__ off) {
  __shared__ int cnt[MOE_MAX_E];
  __shared__ int base[MOE_MAX_E + 1];
  const int tid = threadIdx.x;
  if (tid < MOE_MAX_E) cnt[tid] = 0;
  __syncthreads();
  for (int t = tid; t < T; t += blockDim.x) {
    const float* lg = logits + (size_t)t * E;
    float mx = -INFINITY;
    for (int e = 0; e < E; ++e) mx = fmaxf(mx, lg[e]);
    float sel_v[MOE_MAX_K];
    int sel_i[MOE_MAX_K];
    for (int j = 0; j < k; ++j) {
      sel_v[j] = -INFINITY;
      sel_i[j] = 0;
    }
    for (int e = 0; e < E; ++e) {  // insertion into the running top-k (ties -> lower expert id)
      float v = lg[e];
      int id = e;
      for (int j = 0; j < k; ++j) {
        if (v > sel_v[j]) {
          const float tv = sel_v[j];
          const int ti = sel_i[j];
          sel_v[j] = v;
          sel_i[j] = id;
          v = tv;
          id = ti;
        }
      }
    }
    // softmax restricted to the selected experts == top-k of the full softmax, renormalised
    float den = 0.f;
    for (int j = 0; j < k; ++j) den += __expf(sel_v[j] - mx);
    for (int j = 0; j < k; ++j) {
      topw[(size_t)t * k + j] = __expf(sel_v[j] - mx) / den;
      topi[(size_t)t * k + j] = sel_i[j];
      atomicAdd(&cnt[sel_i[j]], 1);
    }
  }
  __syncthreads();
  if (tid == 0) {
    int acc = 0;
    for (int e = 0; e < E; ++e) {
      base[e] = acc;
      off[e] = acc;
      acc += cnt[e];
    }
    off[E] = acc;
  }
  __syncthreads();
  if (tid < E) cnt[tid] = 0;
  __syncthreads();
  for (int t = tid; t < T; t += blockDim.x) {
    for (int j = 0; j < k; ++j) {
      const int e = topi[(size_t)t * k + j];
      const int pos = base[e] + atomicAdd(&cnt[e], 1);
      slot_of[(size_t)t * k + j] = pos;
      sorted_tok[pos] = t;
    }
  }
}

// DeepSeekMoE routing (HF DeepseekV2TopkRouter / DeepseekV3TopkRouter):
//   score = softmax(logits) (V2) or sigmoid(logits) (V3); choice = score + bias (V3 selection bias)
//   groups: experts in n_group equal groups; keep the topk_group groups ranked by max(choice) (V2
//   group_limited_greedy) or the sum of their two best choices (V3 noaux_tc); top-k experts by choice among
//   the kept groups; weight = score (not choice), optionally renormalised, times routed_scaling_factor.
// Kernel 1: one wave per token (lane l holds experts l, l+64, ..); group statistics from an LDS copy of the
// token's choices; k rounds of a wave argmax; per-expert counts by global atomics.  Kernel 2 (one workgroup):
// exclusive scan of the counts -> expert offsets, slot per (token, j), and the counters reset to zero for
// the next launch (so the graph-captured sequence needs no memset).
constexpr int MOE_DS_MAX_E = 256;
constexpr int MOE_DS_MAX_G = 16;
constexpr int MOE_DS_EPL = MOE_DS_MAX_E / 64;  // experts per lane

__global__ __launch_bounds__(256) void moe_topk_ds_kernel(const float* __restrict__ logits,
                                                          const float* __restrict__ bias, int T, int E, int k,
                                                          int n_group, int topk_group, int method, int sigmoid,
                                                          int norm, float scale, float* __restrict__ topw,
                                                          int32_t* __restrict__ topi, int* __restrict__ cnt) {
  __shared__ float ch_lds[4][MOE_DS_MAX_E];
  __shared__ unsigned keep_lds[4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int t = blockIdx.x * 4 + wave;
  if (t >= T) return;  // wave-uniform; no workgroup barrier below
  const float* lg = logits + (size_t)t * E;
  float sc[MOE_DS_EPL], chv[MOE_DS_EPL];
  float mx = -INFINITY;
#pragma unroll
  for (int i = 0; i < MOE_DS_EPL; ++i) {
    const int e = lane + 64 * i;
    sc[i] = e < E ? lg[e] : -INFINITY;
    mx = fmaxf(mx, sc[i]);
  }
  if (!sigmoid) {
    mx = wave_max(mx);
    float den = 0.f;
#pragma unroll
    for (int i = 0; i < MOE_DS_EPL; ++i) {
      sc[i] = lane + 64 * i < E ? __expf(sc[i] - mx) : 0.f;
      den += sc[i];
    }
    den = wave_sum(den);
#pragma unroll
    for (int i = 0; i < MOE_DS_EPL; ++i) sc[i] /= den;
  } else {
#pragma unroll
    for (int i = 0; i < MOE_DS_EPL; ++i) sc[i] = lane + 64 * i < E ? 1.f / (1.f + __expf(-sc[i])) : 0.f;
  }
#pragma unroll
  for (int i = 0; i < MOE_DS_EPL; ++i) {
    const int e = lane + 64 * i;
    chv[i] = e < E ? sc[i] + (bias != nullptr ? bias[e] : 0.f) : -INFINITY;
    if (e < E) ch_lds[wave][e] = chv[i];
  }
  const int per = E / n_group;
  unsigned keep = 0xffffffffu;
  if (n_group > 1 && topk_group < n_group) {
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    // lane g < n_group: its group's best (V2) or best-two sum (V3) over the LDS copy
    float gsc = -INFINITY;
    if (lane < n_group) {
      float a = -INFINITY, b2 = -INFINITY;
      for (int e = lane * per; e < (lane + 1) * per; ++e) {
        const float v = ch_lds[wave][e];
        if (v > a) {
          b2 = a;
          a = v;
        } else if (v > b2) {
          b2 = v;
        }
      }
      gsc = method == 2 ? a + b2 : a;
    }
    keep = 0;
    for (int j = 0; j < topk_group; ++j) {  // wave argmax over the groups (ties: lower group id)
      float v = (lane < n_group && !(keep >> lane & 1u)) ? gsc : -INFINITY;
      int id = lane;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const float ov = __shfl_xor(v, o, 64);
        const int oi = __shfl_xor(id, o, 64);
        if (ov > v || (ov == v && oi < id)) {
          v = ov;
          id = oi;
        }
      }
      keep |= 1u << id;
    }
  }
#pragma unroll
  for (int i = 0; i < MOE_DS_EPL; ++i) {
    const int e = lane + 64 * i;
    if (e >= E || !(keep >> (e / per) & 1u)) chv[i] = -INFINITY;
  }
  float wsum = 0.f, wj_mine = 0.f;
  int ej_mine = 0;
  for (int j = 0; j < k; ++j) {  // k rounds of a wave argmax over the kept experts (ties: lower expert id)
    float v = -INFINITY;
    int id = 0x7fffffff;
#pragma unroll
    for (int i = 0; i < MOE_DS_EPL; ++i) {
      const int e = lane + 64 * i;
      if (chv[i] > v) {
        v = chv[i];
        id = e;
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(v, o, 64);
      const int oi = __shfl_xor(id, o, 64);
      if (ov > v || (ov == v && oi < id)) {
        v = ov;
        id = oi;
      }
    }
    // the owner lane retires the winner and contributes its score
    float wv = 0.f;
#pragma unroll
    for (int i = 0; i < MOE_DS_EPL; ++i)
      if (lane + 64 * i == id) {
        chv[i] = -INFINITY;
        wv = sc[i];
      }
    wv = wave_sum(wv);
    wsum += wv;
    if (lane == j) {
      wj_mine = wv;
      ej_mine = id;
    }
  }
  const float f = norm ? scale / (wsum + 1e-20f) : scale;
  if (lane < k) {
    topw[(size_t)t * k + lane] = wj_mine * f;
    topi[(size_t)t * k + lane] = ej_mine;
    atomicAdd(cnt + ej_mine, 1);
  }
}

__global__ __launch_bounds__(1024) void moe_slots_kernel(const int32_t* __restrict__ topi, int T, int E, int k,
                                                         int* __restrict__ cnt, int32_t* __restrict__ slot_of,
                                                         int32_t* __restrict__ sorted_tok, int32_t* __restrict__ off) {
  __shared__ int base[MOE_DS_MAX_E + 1];
  __shared__ int cur[MOE_DS_MAX_E];
  const int tid = threadIdx.x;
  if (tid == 0) {
    int acc = 0;
    for (int e = 0; e < E; ++e) {
      base[e] = acc;
      off[e] = acc;
      acc += cnt[e];
    }
    off[E] = acc;
  }
  for (int e = tid; e < E; e += blockDim.x) cur[e] = 0;
  __syncthreads();
  for (int e = tid; e < E; e += blockDim.x) cnt[e] = 0;  // ready for the next launch
  for (int q = tid; q < T * k; q += blockDim.x) {
    const int e = topi[q];
    const int pos = base[e] + atomicAdd(&cur[e], 1);
    slot_of[q] = pos;
    sorted_tok[pos] = q / k;
  }
}

int launch_moe_route_ds(const float* logits, const float* bias, int T, int E, int k, int n_group, int topk_group,
                        int method, bool sigmoid, bool norm, float scale, int* cnt, float* topw, int32_t* topi,
                        int32_t* slot_of, int32_t* sorted_tok, int32_t* off, hipStream_t s) {
  if (E < 1 || E > MOE_DS_MAX_E || k < 1 || k > 64 || n_group < 1 || n_group > MOE_DS_MAX_G || E % n_group != 0 ||
      topk_group < 1 || topk_group > n_group || k > (E / n_group) * topk_group)
    return -1;
  if (T <= 0) return 0;
  moe_topk_ds_kernel<<<(T + 3) / 4, 256, 0, s>>>(logits, bias, T, E, k, n_group, topk_group, method, sigmoid ? 1 : 0,
                                                 norm ? 1 : 0, scale, topw, topi, cnt);
  moe_slots_kernel<<<1, 1024, 0, s>>>(topi, T, E, k, cnt, slot_of, sorted_tok, off);
  return 0;
}

// one thread per 8 hidden columns of one token
__global__ __launch_bounds__(256) void moe_combine_kernel(const float* __restrict__ y,
                                                          const int32_t* __restrict__ slot_of,
                                                          const float* __restrict__ topw, uint16_t* __restrict__ h,
                                                          int T, int k, int D, int S, long ysplit) {
  const long total = (long)T * (D / 8);
  for (long q = blockIdx.x * 256L + threadIdx.x; q < total; q += (long)gridDim.x * 256) {
    const int t = (int)(q / (D / 8));
    const int d = (int)(q % (D / 8)) * 8;
    s16x8 hv = ld16(h + (size_t)t * D + d);
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = bf2f(hv[e]);
    for (int j = 0; j < k; ++j) {
      const float w = topw[(size_t)t * k + j];
      const float* yr = y + (size_t)slot_of[(size_t)t * k + j] * D + d;
      for (int sl = 0; sl < S; ++sl, yr += ysplit) {  // K-slice partial slabs of the grouped down GEMM
        const f32x4 a = *reinterpret_cast<const f32x4*>(yr);
        const f32x4 b = *reinterpret_cast<const f32x4*>(yr + 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          acc[e] += w * a[e];
          acc[4 + e] += w * b[e];
        }
      }
    }
    s16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (short)f2bf(acc[e]);
    st16(h + (size_t)t * D + d, o);
  }
}

// combine + the RMSNorm that follows the MoE block (next layer's input norm / final norm), one
// workgroup per token: h[t] += sum_j w_j y[slot(t, j)] in place, out[t] = rmsnorm(h[t]) * ln_w.  Saves the
// separate norm launch and its re-read of h (a decode step of one token otherwise pays two ~5 us launches).
template <int MAXC>
__global__ __launch_bounds__(256) void moe_combine_norm_kernel(const float* __restrict__ y,
                                                               const int32_t* __restrict__ slot_of,
                                                               const float* __restrict__ topw, uint16_t* __restrict__ h,
                                                               const uint16_t* __restrict__ lnw,
                                                               uint16_t* __restrict__ out, int k, int D, int S,
                                                               long ysplit, float eps) {
  __shared__ float red[4];
  const int t = blockIdx.x, tid = threadIdx.x, nchunk = D >> 3;
  float v[MAXC][8];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < MAXC; ++i) {
    const int c = tid + i * 256;
    if (c >= nchunk) continue;
    const int d = c * 8;
    const s16x8 hv = ld16(h + (size_t)t * D + d);
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = bf2f(hv[e]);
    for (int j = 0; j < k; ++j) {
      const float w = topw[(size_t)t * k + j];
      const float* yr = y + (size_t)slot_of[(size_t)t * k + j] * D + d;
      for (int sl = 0; sl < S; ++sl, yr += ysplit) {
        const f32x4 a = *reinterpret_cast<const f32x4*>(yr);
        const f32x4 b = *reinterpret_cast<const f32x4*>(yr + 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          acc[e] += w * a[e];
          acc[4 + e] += w * b[e];
        }
      }
    }
    s16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      o[e] = (short)f2bf(acc[e]);
      v[i][e] = bf2f(o[e]);  // normalise the stored (bf16) stream, as the unfused path does
      ss += v[i][e] * v[i][e];
    }
    st16(h + (size_t)t * D + d, o);
  }
  ss = wave_sum(ss);
  if ((tid & 63) == 0) red[tid >> 6] = ss;
  __syncthreads();
  const float inv = rsqrtf((red[0] + red[1] + red[2] + red[3]) / (float)D + eps);
#pragma unroll
  for (int i = 0; i < MAXC; ++i) {
    const int c = tid + i * 256;
    if (c >= nchunk) continue;
    const s16x8 wv = ld16(lnw + c * 8);
    s16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (short)f2bf(v[i][e] * inv * bf2f(wv[e]));
    st16(out + (size_t)t * D + c * 8, o);
  }
}

int launch_moe_combine_norm(const float* y, const int32_t* slot_of, const float* topw, uint16_t* h,
                            const uint16_t* lnw, uint16_t* out, int T, int k, int D, int S, long ysplit, float eps,
                            hipStream_t s) {
  if (T <= 0) return 0;
  const int nchunk = D / 8;
  if (D % 8 != 0 || nchunk > 8 * 256) return -1;
#define XOT_MCN(MC) moe_combine_norm_kernel<MC><<<T, 256, 0, s>>>(y, slot_of, topw, h, lnw, out, k, D, S, ysplit, eps)
  if (nchunk <= 256) XOT_MCN(1);
  else if (nchunk <= 512) XOT_MCN(2);
  else if (nchunk <= 1024) XOT_MCN(4);
  else XOT_MCN(8);
#undef XOT_MCN
  return 0;
}

// Router logits in fp32: out[t][e] = x[t] . W[e] (x [T, D] bf16, W [E, D] bf16), one 256-thread workgroup per
// token; W (64 KB for Mixtral) stays in L2 across the workgroups.  Replaces a bf16-output library GEMM plus
// an fp32 cast (two launches, bf16-rounded logits) in front of moe_route.
template <int E>
__global__ __launch_bounds__(256) void router_logits_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ w,
                                                            float* __restrict__ out, int D) {
  __shared__ float red[4][E];
  const int t = blockIdx.x, tid = threadIdx.x;
  float acc[E];
#pragma unroll
  for (int e = 0; e < E; ++e) acc[e] = 0.f;
  const uint16_t* xr = x + (size_t)t * D;
  for (int c = tid; c < D / 8; c += 256) {
    const s16x8 xv = ld16(xr + c * 8);
    float xf[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) xf[j] = bf2f(xv[j]);
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const s16x8 wv = ld16(w + (size_t)e * D + c * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[e] += xf[j] * bf2f(wv[j]);
    }
  }
#pragma unroll
  for (int e = 0; e < E; ++e) {
    float v = acc[e];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if ((tid & 63) == 0) red[tid >> 6][e] = v;
  }
  __syncthreads();
  if (tid < E) out[(size_t)t * E + tid] = red[0][tid] + red[1][tid] + red[2][tid] + red[3][tid];
}

// The same logits on MFMA for the wide routers (DeepSeek: 64 / 160 / 256 experts).  A workgroup takes 16
// tokens x all E = 16 ET experts; its NW waves split K into contiguous slices (decode has only T / 16
// workgroups, so the split is what keeps each wave's dependent chain to a few k iterations).  Per 32-deep
// k step a lane loads its token row's 8 k values (A fragment: row lane & 15, k 8 (lane >> 4)) and each
// expert tile's row (B fragment, same map) from global / L2, U steps at a time with every load issued before
// the MFMAs; the NW partial 16 x E tiles are summed in LDS in wave order (deterministic).  Rows past T
// re-read row T - 1 and are not stored.  Requires D % (128 NW) == 0.
template <int ET, int NW>
__global__ __launch_bounds__(NW * 64) void router_logits_mfma_kernel(const uint16_t* __restrict__ x,
                                                                     const uint16_t* __restrict__ w,
                                                                     float* __restrict__ out, int T, int D) {
  constexpr int E = 16 * ET;
  constexpr int U = ET <= 4 ? 4 : (ET <= 8 ? 2 : 1);  // k steps in flight per iteration (register budget)
  extern __shared__ float red[];                      // [NW][16][E] partial logits
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, c = lane & 15;
  const int t0 = blockIdx.x * 16;
  const int kq = D / NW, kb = wave * kq;
  const uint16_t* xr = x + (size_t)min(t0 + c, T - 1) * D + kb + 8 * g;
  const uint16_t* wr = w + (size_t)c * D + kb + 8 * g;  // + 16 j D for tile j
  f32x4 acc[ET];
#pragma unroll
  for (int j = 0; j < ET; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < kq; k0 += 32 * U) {
    s16x8 a[U], b[U][ET];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      a[u] = ld16(xr + k0 + 32 * u);
#pragma unroll
      for (int j = 0; j < ET; ++j) b[u][j] = ld16(wr + (size_t)16 * j * D + k0 + 32 * u);
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < ET; ++j) acc[j] = mfma16(a[u], b[u][j], acc[j]);
  }
#pragma unroll
  for (int j = 0; j < ET; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) red[(wave * 16 + 4 * g + r) * E + 16 * j + c] = acc[j][r];
  __syncthreads();
  for (int i = threadIdx.x; i < 16 * E; i += NW * 64) {
    float v = 0.f;
#pragma unroll
    for (int q = 0; q < NW; ++q) v += red[q * 16 * E + i];
    const int t = t0 + i / E;
    if (t < T) out[(size_t)t * E + i % E] = v;
  }
}

template <int ET, int NW>
static void router_mfma_launch(const uint16_t* x, const uint16_t* w, float* out, int T, int D, hipStream_t s) {
  router_logits_mfma_kernel<ET, NW><<<(T + 15) / 16, NW * 64, NW * 16 * 16 * ET * 4, s>>>(x, w, out, T, D);
}

int launch_router_logits(const uint16_t* x, const uint16_t* w, float* out, int T, int E, int D, hipStream_t s) {
  if (T <= 0) return 0;
  if (D % 8 != 0) return -1;
  if (E >= 32 && D % 512 == 0) {
    const bool w8 = E <= 128 && D % 1024 == 0;  // 8 waves (LDS 8 x 16 x E x 4 B <= 64 KB) when K allows
#define XOT_RL(ETV)                                                        \
  do {                                                                     \
    if (w8) router_mfma_launch<ETV, 8>(x, w, out, T, D, s);               \
    else router_mfma_launch<ETV, 4>(x, w, out, T, D, s);                   \
    return 0;                                                              \
  } while (0)
    switch (E) {
      case 32: XOT_RL(2);
      case 64: XOT_RL(4);
      case 128: XOT_RL(8);
      case 160: XOT_RL(10);
      case 256: XOT_RL(16);
      default: break;
    }
#undef XOT_RL
  }
  switch (E) {
    case 8: router_logits_kernel<8><<<T, 256, 0, s>>>(x, w, out, D); return 0;
    case 16: router_logits_kernel<16><<<T, 256, 0, s>>>(x, w, out, D); return 0;
    case 4: router_logits_kernel<4><<<T, 256, 0, s>>>(x, w, out, D); return 0;
    default: return -1;
  }
}

void launch_moe_route(const float* logits, int T, int E, int k, float* topw, int32_t* topi, int32_t* slot_of,
                      int32_t* sorted_tok, int32_t* off, hipStream_t s) {
  moe_route_kernel<<<1, 1024, 0, s>>>(logits, T, E, k, topw, topi, slot_of, sorted_tok, off);
}

void launch_moe_combine(const float* y, const int32_t* slot_of, const float* topw, uint16_t* h, int T, int k, int D,
                        int S, long ysplit, hipStream_t s) {
  const long chunks = (long)T * (D / 8);
  int blocks = (int)((chunks + 255) / 256);
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) return;
  moe_combine_kernel<<<blocks, 256, 0, s>>>(y, slot_of, topw, h, T, k, D, S, ysplit);
}

}  // namespace xot

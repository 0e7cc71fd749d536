// On-device token sampling: one 1024-thread workgroup per row of logits.
//
// Semantics follow the reference's torchtune `sample` (xotorch/inference/torch/sharded_inference_engine.py:208-228):
//   logits / max(temp, 1e-5) -> keep values >= the k-th largest (ties kept) -> softmax ->
//   argmax(probs / q), q ~ Exponential(1)
// which is the exponential-race form of categorical sampling.  Here it is computed as
//   argmax_{i: logit_i >= kth} ( logit_i / T - log(-log u_i) ),  u_i = counter-hash(seed, offset, row, i)
// so no softmax is materialised and nothing leaves the device (the reference does D2H -> H2D -> D2H
// per token).  The k-th largest logit is found exactly by a 4-pass 8-bit radix select on the
// order-preserving uint32 image of the floats.  temp <= 1e-5 (the default --default-temp 0.0) or
// top_k == 1 takes the argmax path (first index on ties, as torch.argmax).
#include "common.h"
#include "kernels.h"

namespace xot {

__device__ __forceinline__ uint32_t fkey(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ void argmax_combine(float& v, int& i, float v2, int i2) {
  if (v2 > v || (v2 == v && i2 < i)) {
    v = v2;
    i = i2;
  }
}

// Radix-select step, run by wave 0: find the bin holding the krem-th largest key (bins scanned from
// 255 down) with a wave suffix scan instead of a 256-long dependent LDS chain (which alone cost
// ~25 us per row).  Writes the refined prefix and the remaining rank to shv[0], shv[1].
__device__ __forceinline__ void pick_bin(const int* hist, uint32_t krem, uint32_t prefix, int shift, uint32_t* shv) {
  const int l = threadIdx.x;  // 0..63
  const int b0 = 255 - 4 * l;
  const int c0 = hist[b0], c1 = hist[b0 - 1], c2 = hist[b0 - 2], c3 = hist[b0 - 3];
  const int sum = c0 + c1 + c2 + c3;
  int incl = sum;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(incl, o, 64);
    if (l >= o) incl += t;
  }
  const int excl = incl - sum;
  const bool hit = (uint32_t)excl < krem && krem <= (uint32_t)incl;
  const unsigned long long m = __ballot(hit);
  const int L = m ? __ffsll((long long)m) - 1 : 63;
  if (l == L) {
    const int cs[4] = {c0, c1, c2, c3};
    uint32_t cum = excl;
    int bin = b0 - 3;
    for (int j = 0; j < 4; ++j) {
      if (b0 - j == 0 || cum + (uint32_t)cs[j] >= krem) {
        bin = b0 - j;
        break;
      }
      cum += cs[j];
    }
    shv[0] = prefix | ((uint32_t)bin << shift);
    shv[1] = krem - cum;
  }
}

__global__ __launch_bounds__(1024) void sample_kernel(const float* __restrict__ logits, long ld, int V,
                                                      const float* __restrict__ temps, int top_k,
                                                      const int64_t* __restrict__ seed_off,
                                                      int32_t* __restrict__ out) {
  __shared__ int hist[256];
  __shared__ float rv[16];
  __shared__ int ri[16];
  __shared__ uint32_t shv1[2];
  const int row = blockIdx.x, tid = threadIdx.x;
  const float* x = logits + (size_t)row * ld;
  const float temp = temps[row];
  const bool greedy = temp <= 1e-5f || top_k == 1;

  uint32_t thresh = 0;  // keys >= thresh are eligible
  if (!greedy && top_k > 0 && top_k < V) {
    uint32_t prefix = 0, krem = (uint32_t)top_k;
    for (int pass = 0; pass < 4; ++pass) {
      const int shift = 24 - 8 * pass;
      const uint32_t hmask = pass == 0 ? 0u : (0xFFFFFFFFu << (shift + 8));
      for (int i = tid; i < 256; i += 1024) hist[i] = 0;
      __syncthreads();
      for (int i = tid; i < V; i += 1024) {
        const uint32_t k = fkey(x[i]);
        if ((k & hmask) == prefix) atomicAdd(&hist[(k >> shift) & 255], 1);
      }
      __syncthreads();
      if (tid < 64) pick_bin(hist, krem, prefix, shift, shv1);
      __syncthreads();
      prefix = shv1[0];
      krem = shv1[1];
      __syncthreads();
    }
    thresh = prefix;  // exact key of the k-th largest value
  }

  const float invt = greedy ? 1.f : 1.f / fmaxf(temp, 1e-5f);
  const uint64_t seed = (uint64_t)seed_off[0], off = (uint64_t)seed_off[1];
  const uint64_t base = splitmix64(seed ^ splitmix64(off * 0x632be59bd9b4e019ull + (uint64_t)row));
  float best = -INFINITY;
  int bidx = 0x7fffffff;
  for (int i = tid; i < V; i += 1024) {
    const float v = x[i];
    float s;
    if (greedy) {
      s = v;
    } else {
      if (fkey(v) < thresh) continue;
      const uint64_t h = splitmix64(base + (uint64_t)i);
      const float u = ((float)(h >> 40) + 0.5f) * (1.0f / 16777216.0f);  // (0,1)
      s = v * invt - __logf(-__logf(u));
    }
    argmax_combine(best, bidx, s, i);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float v2 = __shfl_xor(best, o, 64);
    const int i2 = __shfl_xor(bidx, o, 64);
    argmax_combine(best, bidx, v2, i2);
  }
  if ((tid & 63) == 0) {
    rv[tid >> 6] = best;
    ri[tid >> 6] = bidx;
  }
  __syncthreads();
  if (tid == 0) {
    float bv = rv[0];
    int bi = ri[0];
    for (int w = 1; w < 16; ++w) argmax_combine(bv, bi, rv[w], ri[w]);
    out[row] = bi >= V ? 0 : bi;
  }
}

// ---------------------------------------------------------------------------- small batches
// With few rows a single workgroup per row leaves the chip idle and is latency-bound (~150 us for
// one 128k-vocab row).  Split each row over SG chunk workgroups: stage 1 keeps every chunk's top-k
// (key, index) candidates (for greedy rows: the chunk argmax); stage 2, one workgroup per row,
// selects the global k-th largest among the SG*k candidates and runs the same exponential race on
// the eligible ones.  Every element >= the global k-th largest is in its chunk's top-k, so both
// paths pick the same token for the same (seed, offset) except under exact float ties at the cut.
constexpr int SG = 64;       // chunks per row
constexpr int SK = 64;       // max top_k on this path
constexpr int SCH = 2048;    // max chunk length (V <= SG * SCH)

// block-wide 4-pass radix select over n keys in LDS: the key of the krem-th largest
__device__ uint32_t radix_kth(const uint32_t* keys, int n, uint32_t krem, int* hist, uint32_t* shv) {
  const int tid = threadIdx.x;
  uint32_t prefix = 0;
  for (int pass = 0; pass < 4; ++pass) {
    const int shift = 24 - 8 * pass;
    const uint32_t hmask = pass == 0 ? 0u : (0xFFFFFFFFu << (shift + 8));
    for (int i = tid; i < 256; i += blockDim.x) hist[i] = 0;
    __syncthreads();
    for (int i = tid; i < n; i += blockDim.x) {
      const uint32_t k = keys[i];
      if ((k & hmask) == prefix) atomicAdd(&hist[(k >> shift) & 255], 1);
    }
    __syncthreads();
    if (tid < 64) pick_bin(hist, krem, prefix, shift, shv);
    __syncthreads();
    prefix = shv[0];
    krem = shv[1];
    __syncthreads();
  }
  return prefix;
}

__global__ __launch_bounds__(256) void sample_stage1_kernel(const float* __restrict__ logits, long ld, int V,
                                                            const float* __restrict__ temps, int top_k,
                                                            uint32_t* __restrict__ cand_key,
                                                            int32_t* __restrict__ cand_idx) {
  __shared__ uint32_t keys[SCH];
  __shared__ int hist[256];
  __shared__ uint32_t shv[2];
  __shared__ int cnt;
  __shared__ float rv[4];
  __shared__ int ri[4];
  const int chunk = blockIdx.x, row = blockIdx.y, tid = threadIdx.x;
  const int len = (V + SG - 1) / SG, beg = chunk * len, n = max(0, min(len, V - beg));
  const float* x = logits + (size_t)row * ld + beg;
  uint32_t* ck = cand_key + ((size_t)row * SG + chunk) * SK;
  int32_t* ci = cand_idx + ((size_t)row * SG + chunk) * SK;
  const bool greedy = temps[row] <= 1e-5f || top_k == 1;
  if (greedy) {  // chunk argmax -> candidate slot 0
    float best = -INFINITY;
    int bidx = 0x7fffffff;
    for (int i = tid; i < n; i += 256) argmax_combine(best, bidx, x[i], beg + i);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float v2 = __shfl_xor(best, o, 64);
      const int i2 = __shfl_xor(bidx, o, 64);
      argmax_combine(best, bidx, v2, i2);
    }
    if ((tid & 63) == 0) {
      rv[tid >> 6] = best;
      ri[tid >> 6] = bidx;
    }
    __syncthreads();
    if (tid == 0) {
      float bv = rv[0];
      int bi = ri[0];
      for (int w = 1; w < 4; ++w) argmax_combine(bv, bi, rv[w], ri[w]);
      ck[0] = fkey(bv);
      ci[0] = bi;
    }
    return;
  }
  for (int i = tid; i < n; i += 256) keys[i] = fkey(x[i]);
  if (tid == 0) cnt = 0;
  __syncthreads();
  const int kk = min(top_k, n);
  const uint32_t th = kk > 0 ? radix_kth(keys, n, (uint32_t)kk, hist, shv) : 0xFFFFFFFFu;
  // emit the chunk's top-kk (keys > th first, then ties at th up to kk)
  for (int i = tid; i < n; i += 256)
    if (keys[i] > th) {
      const int p = atomicAdd(&cnt, 1);
      ck[p] = keys[i];
      ci[p] = beg + i;
    }
  __syncthreads();
  for (int i = tid; i < n; i += 256)
    if (keys[i] == th) {
      const int p = atomicAdd(&cnt, 1);
      if (p < kk) {
        ck[p] = keys[i];
        ci[p] = beg + i;
      }
    }
  __syncthreads();
  for (int p = min(cnt, kk) + tid; p < SK; p += 256) {  // unused slots
    ck[p] = 0;
    ci[p] = -1;
  }
}

__global__ __launch_bounds__(256) void sample_stage2_kernel(const float* __restrict__ temps, int top_k,
                                                            const int64_t* __restrict__ seed_off,
                                                            const uint32_t* __restrict__ cand_key,
                                                            const int32_t* __restrict__ cand_idx, int V,
                                                            int32_t* __restrict__ out) {
  __shared__ uint32_t keys[SG * SK];
  __shared__ int hist[256];
  __shared__ uint32_t shv[2];
  __shared__ float rv[4];
  __shared__ int ri[4];
  const int row = blockIdx.x, tid = threadIdx.x;
  const uint32_t* ck = cand_key + (size_t)row * SG * SK;
  const int32_t* ci = cand_idx + (size_t)row * SG * SK;
  const float temp = temps[row];
  const bool greedy = temp <= 1e-5f || top_k == 1;
  const int n = SG * SK;
  for (int i = tid; i < n; i += 256) keys[i] = (greedy && (i % SK) != 0) ? 0u : (ci[i] < 0 ? 0u : ck[i]);
  // (unused slots hold key 0, below every real key, so they never reach the top-k)
  __syncthreads();
  uint32_t th = 0;
  if (!greedy) th = radix_kth(keys, n, (uint32_t)top_k, hist, shv);
  const float invt = greedy ? 1.f : 1.f / fmaxf(temp, 1e-5f);
  const uint64_t seed = (uint64_t)seed_off[0], off = (uint64_t)seed_off[1];
  const uint64_t base = splitmix64(seed ^ splitmix64(off * 0x632be59bd9b4e019ull + (uint64_t)row));
  float best = -INFINITY;
  int bidx = 0x7fffffff;
  for (int i = tid; i < n; i += 256) {
    const int idx = ci[i];
    if (idx < 0 || keys[i] < th || (greedy && (i % SK) != 0)) continue;
    // invert fkey to recover the logit
    const uint32_t k = keys[i];
    const float v = __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
    float sc;
    if (greedy) {
      sc = v;
    } else {
      const uint64_t h = splitmix64(base + (uint64_t)idx);
      const float u = ((float)(h >> 40) + 0.5f) * (1.0f / 16777216.0f);
      sc = v * invt - __logf(-__logf(u));
    }
    argmax_combine(best, bidx, sc, idx);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float v2 = __shfl_xor(best, o, 64);
    const int i2 = __shfl_xor(bidx, o, 64);
    argmax_combine(best, bidx, v2, i2);
  }
  if ((tid & 63) == 0) {
    rv[tid >> 6] = best;
    ri[tid >> 6] = bidx;
  }
  __syncthreads();
  if (tid == 0) {
    float bv = rv[0];
    int bi = ri[0];
    for (int w = 1; w < 4; ++w) argmax_combine(bv, bi, rv[w], ri[w]);
    out[row] = bi >= V ? 0 : bi;
  }
}

// ---------------------------------------------------------------------------- large batches
// One 1024-thread workgroup per row, two streaming passes instead of five: pass 1 takes every thread's
// maximum; the top_k-th largest of those 1024 maxima is a lower bound t0 of the row's top_k-th largest
// logit (they are top_k distinct elements), so pass 2 keeps only the (typically a few dozen) elements
// >= t0 as LDS candidates; the exact k-th largest is radix-selected among them and the same
// exponential race as sample_kernel runs on the eligible ones -> the same token for the same
// (seed, offset).  Candidate overflow (massive ties) falls back to the exact 4-pass radix over the row.
constexpr int FCAP = 4096;

// CAND: instead of sampling, write each row's top_k (value, index) candidates to cval / cidx_o [B][kc]
// (ties at the cut trimmed to top_k; unused slots -inf / -1) -- one vocab slice's share of a sampler
// that runs elsewhere (parallel/pipeline.py: LM head split between the last and the first ring stage).
template <bool CAND>
__global__ __launch_bounds__(1024) void sample_fast_kernel(const float* __restrict__ logits, long ld, int V,
                                                           const float* __restrict__ temps, int top_k,
                                                           const int64_t* __restrict__ seed_off,
                                                           int32_t* __restrict__ out, float* __restrict__ cval,
                                                           int32_t* __restrict__ cidx_o, int kc) {
  __shared__ uint32_t ckey[FCAP];
  __shared__ int cidx[FCAP];
  __shared__ uint32_t mkeys[1024];
  __shared__ int hist[256];
  __shared__ uint32_t shv[2];
  __shared__ int cnt;
  __shared__ float rv[16];
  __shared__ int ri[16];
  const int row = blockIdx.x, tid = threadIdx.x;
  const float* x = logits + (size_t)row * ld;
  const float4* x4 = reinterpret_cast<const float4*>(x);
  const int V4 = V >> 2;
  const float temp = CAND ? 1.f : temps[row];
  const bool greedy = !CAND && (temp <= 1e-5f || top_k == 1);
  const bool filter = CAND || (!greedy && top_k > 0 && top_k < V);

  // pass 1: per-thread max (and first argmax for greedy rows)
  float best = -INFINITY;
  int bidx = 0x7fffffff;
  for (int i = tid; i < V4; i += 1024) {
    const float4 v = x4[i];
    argmax_combine(best, bidx, v.x, 4 * i);
    argmax_combine(best, bidx, v.y, 4 * i + 1);
    argmax_combine(best, bidx, v.z, 4 * i + 2);
    argmax_combine(best, bidx, v.w, 4 * i + 3);
  }
  auto block_argmax = [&](float bv, int bi) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float v2 = __shfl_xor(bv, o, 64);
      const int i2 = __shfl_xor(bi, o, 64);
      argmax_combine(bv, bi, v2, i2);
    }
    if ((tid & 63) == 0) {
      rv[tid >> 6] = bv;
      ri[tid >> 6] = bi;
    }
    __syncthreads();
    if (tid == 0) {
      float b2 = rv[0];
      int i2 = ri[0];
      for (int w = 1; w < 16; ++w) argmax_combine(b2, i2, rv[w], ri[w]);
      out[row] = i2 >= V ? 0 : i2;
    }
  };
  if (greedy) {
    block_argmax(best, bidx);
    return;
  }

  uint32_t th = 0;
  int n = 0;
  bool use_cand = false;
  if (filter) {
    mkeys[tid] = bidx < V ? fkey(best) : 0u;
    if (tid == 0) cnt = 0;
    __syncthreads();
    const uint32_t t0 = radix_kth(mkeys, 1024, (uint32_t)min(top_k, 1024), hist, shv);
    // pass 2: candidates >= t0
    for (int i = tid; i < V4; i += 1024) {
      const float4 v = x4[i];
      const float e[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (fkey(e[j]) >= t0) {
          const int p = atomicAdd(&cnt, 1);
          if (p < FCAP) {
            ckey[p] = fkey(e[j]);
            cidx[p] = 4 * i + j;
          }
        }
    }
    __syncthreads();
    n = cnt;
    use_cand = n <= FCAP;
    if (use_cand) {
      th = radix_kth(ckey, n, (uint32_t)top_k, hist, shv);
    } else {  // exact radix over the whole row
      uint32_t prefix = 0, krem = (uint32_t)top_k;
      for (int pass = 0; pass < 4; ++pass) {
        const int shift = 24 - 8 * pass;
        const uint32_t hmask = pass == 0 ? 0u : (0xFFFFFFFFu << (shift + 8));
        for (int i = tid; i < 256; i += 1024) hist[i] = 0;
        __syncthreads();
        for (int i = tid; i < V; i += 1024) {
          const uint32_t k = fkey(x[i]);
          if ((k & hmask) == prefix) atomicAdd(&hist[(k >> shift) & 255], 1);
        }
        __syncthreads();
        if (tid < 64) pick_bin(hist, krem, prefix, shift, shv);
        __syncthreads();
        prefix = shv[0];
        krem = shv[1];
        __syncthreads();
      }
      th = prefix;
    }
  }

  if constexpr (CAND) {
    __shared__ int ecnt;
    if (tid == 0) ecnt = 0;
    __syncthreads();
    float* cv = cval + (size_t)row * kc;
    int32_t* ci = cidx_o + (size_t)row * kc;
    auto emit = [&](uint32_t k, int i, bool tie) {
      const int p = atomicAdd(&ecnt, 1);
      if (!tie || p < top_k) {
        cv[p] = __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
        ci[p] = i;
      }
    };
    for (int tie = 0; tie < 2; ++tie) {  // keys above the cut (fewer than top_k), then ties at the cut
      if (use_cand) {
        for (int p = tid; p < n; p += 1024)
          if (tie ? ckey[p] == th : ckey[p] > th) emit(ckey[p], cidx[p], tie);
      } else {
        for (int i = tid; i < V; i += 1024) {
          const uint32_t k = fkey(x[i]);
          if (tie ? k == th : k > th) emit(k, i, tie);
        }
      }
      __syncthreads();
    }
    for (int p = min(ecnt, top_k) + tid; p < kc; p += 1024) {
      cv[p] = -INFINITY;
      ci[p] = -1;
    }
    return;
  }

  const float invt = 1.f / fmaxf(temp, 1e-5f);
  const uint64_t seed = (uint64_t)seed_off[0], off = (uint64_t)seed_off[1];
  const uint64_t base = splitmix64(seed ^ splitmix64(off * 0x632be59bd9b4e019ull + (uint64_t)row));
  auto race = [&](float v, int i) {
    const uint64_t h = splitmix64(base + (uint64_t)i);
    const float u = ((float)(h >> 40) + 0.5f) * (1.0f / 16777216.0f);  // (0,1)
    return v * invt - __logf(-__logf(u));
  };
  best = -INFINITY;
  bidx = 0x7fffffff;
  if (use_cand) {
    for (int p = tid; p < n; p += 1024) {
      const uint32_t k = ckey[p];
      if (k < th) continue;
      const float v = __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
      argmax_combine(best, bidx, race(v, cidx[p]), cidx[p]);
    }
  } else {
    for (int i = tid; i < V; i += 1024) {
      const float v = x[i];
      if (fkey(v) < th) continue;
      argmax_combine(best, bidx, race(v, i), i);
    }
  }
  block_argmax(best, bidx);
}

void launch_sample(const float* logits, long ld, int B, int V, const float* temps, int top_k,
                   const int64_t* seed_off, int32_t* out, uint32_t* cand_key, int32_t* cand_idx, hipStream_t s,
                   int algo) {
  if (B <= 0) return;
  // algo: -1 auto, 0 one workgroup per row (5 passes), 1 chunk candidates + merge, 2 two-pass candidate
  // filter (1 and 2 where the shape allows them)
  const bool can = cand_key != nullptr && top_k > 0 && top_k <= SK && V <= SG * SCH && V >= SG * SK;
  const bool fast = (algo == 2 || algo < 0) && V % 4 == 0 && ld % 4 == 0 && ((uintptr_t)logits & 15) == 0 &&
                    top_k <= 1024;
  const bool split = !fast && can && (algo == 1 || (algo < 0 && B < 64));
  if (fast) {  // tools/bench_sample.py: B = 512 297 -> 79 us, B = 1 33 -> 31 us (128k vocab, top-k 35)
    sample_fast_kernel<false><<<B, 1024, 0, s>>>(logits, ld, V, temps, top_k, seed_off, out, nullptr, nullptr, 0);
    return;
  }
  if (split) {
    sample_stage1_kernel<<<dim3(SG, B), 256, 0, s>>>(logits, ld, V, temps, top_k, cand_key, cand_idx);
    sample_stage2_kernel<<<B, 256, 0, s>>>(temps, top_k, seed_off, cand_key, cand_idx, V, out);
    return;
  }
  sample_kernel<<<B, 1024, 0, s>>>(logits, ld, V, temps, top_k, seed_off, out);
}

int launch_topk_cand(const float* logits, long ld, int B, int V, int top_k, float* cval, int32_t* cidx, int kc,
                     hipStream_t s) {
  if (B <= 0) return 0;
  if (top_k < 1 || top_k > kc || top_k >= V || V % 4 != 0 || ld % 4 != 0 || ((uintptr_t)logits & 15) != 0) return -1;
  sample_fast_kernel<true><<<B, 1024, 0, s>>>(logits, ld, V, nullptr, top_k, nullptr, nullptr, cval, cidx, kc);
  return 0;
}

}  // namespace xot

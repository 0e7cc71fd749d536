#include "hip/hip_runtime.h"
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

__global__ __launch_bounds__(1024) void sample_kernel(const float* __restrict__ logits, long ld, int V,
                                                      const float* __restrict__ temps, int top_k,
                                                      const int64_t* __restrict__ seed_off,
                                                      int32_t* __restrict__ out) {
  __shared__ int hist[256];
  __shared__ float rv[16];
  __shared__ int ri[16];
  __shared__ uint32_t sh_prefix, sh_krem;
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
      if (tid == 0) {
        uint32_t cum = 0;
        int bin = 255;
        for (; bin > 0; --bin) {
          if (cum + (uint32_t)hist[bin] >= krem) break;
          cum += hist[bin];
        }
        sh_prefix = prefix | ((uint32_t)bin << shift);
        sh_krem = krem - cum;
      }
      __syncthreads();
      prefix = sh_prefix;
      krem = sh_krem;
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

void launch_sample(const float* logits, long ld, int B, int V, const float* temps, int top_k,
                   const int64_t* seed_off, int32_t* out, hipStream_t s) {
  if (B <= 0) return;
 hipLaunchKernelGGL(( sample_kernel), dim3(B), dim3(1024), 0, s, logits, ld, V, temps, top_k, seed_off, out);
}

}  // namespace xot

// Shared pieces of the GEMM kernels: epilogue kinds and the split-K slab reduction.
#pragma once
#include "common.h"

namespace xot {

enum { EPI_NONE = 0, EPI_RESID = 1, EPI_SILU = 2 };

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) void* glb_ptr_t;

// one LDS-DMA wave instruction: lane l copies 16 B from its own global address to lds_base + 16*l
template <int AUX = 0>
__device__ __forceinline__ void glds16(const void* g, void* lds_base) {
  __builtin_amdgcn_global_load_lds((glb_ptr_t)g, (lds_ptr_t)lds_base, 16, 0, AUX);
}

// wait until at most N of this wave's vector-memory operations (loads, LDS-DMA, stores) are in flight
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// the same for a wave-uniform runtime count 0 <= n <= N (a chain of scalar compares; n clamped to N)
template <int N>
__device__ __forceinline__ void wait_vm_upto(int n) {
  if constexpr (N == 0) {
    wait_vm<0>();
  } else {
    if (n >= N) wait_vm<N>();
    else wait_vm_upto<N - 1>(n);
  }
}

// Sum the S fp32 slabs of one output row at 8 output columns [o, o+8) and apply the epilogue.
// wsrow = slab 0 of this row (slabs are sstride floats apart); rrow / yrow = this row of R / Y.
template <int EPI, bool OUT_F32>
__device__ __forceinline__ void splitk_out8(const float* __restrict__ wsrow, size_t sstride, int S, int o,
                                            const uint16_t* __restrict__ bias, const uint16_t* __restrict__ rrow,
                                            void* __restrict__ yrow) {
  float v[8];
  if constexpr (EPI == EPI_SILU) {
    const int j = o >> 4, w = o & 15;
    float gs[8], us[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) gs[e] = us[e] = 0.f;
    for (int s = 0; s < S; ++s) {
      const float* row = wsrow + s * sstride;
      const f32x4 g0 = *reinterpret_cast<const f32x4*>(row + 32 * j + w);
      const f32x4 g1 = *reinterpret_cast<const f32x4*>(row + 32 * j + w + 4);
      const f32x4 u0 = *reinterpret_cast<const f32x4*>(row + 32 * j + 16 + w);
      const f32x4 u1 = *reinterpret_cast<const f32x4*>(row + 32 * j + 16 + w + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        gs[e] += g0[e];
        gs[e + 4] += g1[e];
        us[e] += u0[e];
        us[e + 4] += u1[e];
      }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float bg = bias ? bf2f(bias[32 * j + w + e]) : 0.f, bu = bias ? bf2f(bias[32 * j + 16 + w + e]) : 0.f;
      v[e] = silu(gs[e] + bg) * (us[e] + bu);
    }
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = 0.f;
    for (int s = 0; s < S; ++s) {
      const float* row = wsrow + s * sstride + o;
      const f32x4 a = *reinterpret_cast<const f32x4*>(row), b = *reinterpret_cast<const f32x4*>(row + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] += a[e];
        v[e + 4] += b[e];
      }
    }
    if (bias != nullptr) {
      const s16x8 bb = ld16(bias + o);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += bf2f(bb[e]);
    }
    if constexpr (EPI == EPI_RESID) {
      const s16x8 rr = ld16(rrow + o);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += bf2f(rr[e]);
    }
  }
  if constexpr (OUT_F32) {
    float* y = reinterpret_cast<float*>(yrow) + o;
    *reinterpret_cast<f32x4*>(y) = f32x4{v[0], v[1], v[2], v[3]};
    *reinterpret_cast<f32x4*>(y + 4) = f32x4{v[4], v[5], v[6], v[7]};
  } else {
    s16x8 out;
#pragma unroll
    for (int e = 0; e < 8; ++e) out[e] = (short)f2bf(v[e]);
    st16(reinterpret_cast<uint16_t*>(yrow) + o, out);
  }
}

// Sum S fp32 slabs [S][M][N] and apply the epilogue.  One thread per 8 output columns.
template <int EPI, bool OUT_F32>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ ws, int S, int M, int N,
                                                            const uint16_t* __restrict__ bias,
                                                            const uint16_t* __restrict__ R, int ldr,
                                                            void* __restrict__ Yv, int ldy) {
  const int ncol = EPI == EPI_SILU ? N / 2 : N;
  const long total = (long)M * (ncol / 8);
  for (long t = blockIdx.x * 256L + threadIdx.x; t < total; t += (long)gridDim.x * 256) {
    const int m = (int)(t / (ncol / 8));
    const int o = (int)(t % (ncol / 8)) * 8;
    void* yrow = OUT_F32 ? (void*)(reinterpret_cast<float*>(Yv) + (size_t)m * ldy)
                         : (void*)(reinterpret_cast<uint16_t*>(Yv) + (size_t)m * ldy);
    splitk_out8<EPI, OUT_F32>(ws + (size_t)m * N, (size_t)M * N, S, o, bias,
                              EPI == EPI_RESID ? R + (size_t)m * ldr : nullptr, yrow);
  }
}

}  // namespace xot

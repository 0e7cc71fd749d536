// Shared device helpers for the CDNA4 (gfx950) kernel library.
//
// Everything here is written for wave64 + MFMA on MI355X: bf16 is carried as raw
// 16-bit storage and widened to fp32 for arithmetic, memory traffic is 16 B per
// lane (8 bf16) wherever the layout allows, and the matrix work goes through
// __builtin_amdgcn_mfma_f32_16x16x32_bf16 (16x16 output tile, K=32 per issue).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

namespace xot {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int WAVE = 64;

__device__ __forceinline__ float bf2f(uint16_t u) { return __uint_as_float(((uint32_t)u) << 16); }
__device__ __forceinline__ float bf2f(short s) { return bf2f((uint16_t)s); }
__device__ __forceinline__ uint16_t f2bf(float f) {
  __hip_bfloat16 h = __float2bfloat16(f);
  return __builtin_bit_cast(uint16_t, h);
}

// 16x16x32 bf16 MFMA.  Operand maps (lane l, j = 0..7):
//   A[row = l&15][k = 8*(l>>4) + j],  B[k = 8*(l>>4) + j][col = l&15]
//   C/D: col = l&15, row = 4*(l>>4) + reg
// Any permutation of k applied identically to A and B leaves the product unchanged;
// the kernels use that to make each lane's operand bytes contiguous in memory.
__device__ __forceinline__ f32x4 mfma16(const s16x8& a, const s16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a),
                                                 __builtin_bit_cast(bf16x8_t, b), c, 0, 0, 0);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
// reductions across the 16 lanes that share (l>>4)
__device__ __forceinline__ float group16_sum(float v) {
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float group16_max(float v) {
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

__device__ __forceinline__ s16x8 ld16(const void* p) { return *reinterpret_cast<const s16x8*>(p); }
// non-temporal 16-B load (global_load_dwordx4 ... nt): bytes read once per kernel (KV pages in decode)
__device__ __forceinline__ s16x8 ld16nt(const void* p) {
  return __builtin_nontemporal_load(reinterpret_cast<const s16x8*>(p));
}
__device__ __forceinline__ void st16(void* p, const s16x8& v) { *reinterpret_cast<s16x8*>(p) = v; }

__device__ __forceinline__ float silu(float x) { return x / (1.0f + __expf(-x)); }

// Paged V cache: a 64-key page of one KV head is stored chunk-major, 8 chunks of 8 keys, each chunk [Dh][8]:
// element offset of (key, d) inside the page.  Readers (the attention kernels) load 8 consecutive keys of one dim
// as one 16-B run; a writer's token fills 2 B in each of Dh 16-B runs packed 8 to a 128-B line.
__host__ __device__ __forceinline__ int v_page_off(int key, int d, int Dh) { return ((key >> 3) * Dh + d) * 8 + (key & 7); }

}  // namespace xot

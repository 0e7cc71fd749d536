// Infinity-Cache (MALL) warm-up of a weight that the next GEMM will stream.
//
// Batch-1 decode leaves HBM idle while its short latency-bound kernels run (RoPE + KV write, attention,
// partition merge, reduce + RMSNorm: ~26 us of a 108 us Llama-3-8B layer).  Launched on a side stream in
// that window, this kernel reads the next projection's weight once so the 256 MiB die-level cache holds it;
// the GEMM then streams it from the cache instead of HBM.  Pure reads: the loaded words are folded into one
// value per lane that is stored (vector store, one dword) only in the practically impossible case that it
// equals `sentinel`, which keeps the loads alive without a data-dependent output.
#include "common.h"
#include "kernels.h"

namespace xot {

__global__ __launch_bounds__(256) void mall_prefetch_kernel(const u32x4* __restrict__ p, long n16,
                                                            uint32_t sentinel, uint32_t* __restrict__ sink) {
  constexpr int U = 8;  // independent 16-B loads in flight per lane
  const long stride = (long)gridDim.x * 256;
  long i = (long)blockIdx.x * 256 + threadIdx.x;
  uint32_t acc = 0;
  for (; i + (U - 1) * stride < n16; i += U * stride) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = p[i + u * stride];
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u][0] ^ v[u][1] ^ v[u][2] ^ v[u][3];
  }
  for (; i < n16; i += stride) {
    const u32x4 v = p[i];
    acc ^= v[0] ^ v[1] ^ v[2] ^ v[3];
  }
  if (acc == sentinel) sink[threadIdx.x] = acc;
}

void launch_mall_prefetch(const void* p, size_t bytes, int wgs, uint32_t* sink, hipStream_t s) {
  const long n16 = (long)(bytes / 16);
  if (n16 <= 0) return;
  const long need = (n16 + 256 * 8 - 1) / (256 * 8);
  const int grid = (int)(need < wgs ? need : wgs);
  mall_prefetch_kernel<<<grid, 256, 0, s>>>(reinterpret_cast<const u32x4*>(p), n16, 0x9e3779b9u, sink);
}

}  // namespace xot

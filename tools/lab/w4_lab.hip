// LAB harness (not shipped): times the production four-wave tile (csrc/gemm_w4.hip, compiled here with the -D
// knobs of a variant) on one shape, weights rotated through >= 1 GB (HBM-cold as in a forward pass).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DVARIANT='"name"' [-DW4_XAUX=.. -DW4_WAUX=..] -I<csrc> w4_lab.hip
//   ./w4_lab M N K [iters] [group_m]   -> one JSON line {variant, M, N, K, group_m, us, pflops}
#include "../../xotorch_support_jetson_amd/csrc/gemm_w4.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

#ifndef VARIANT
#define VARIANT "base"
#endif

#define CK(x)                                                          \
  do {                                                                 \
    hipError_t e_ = (x);                                               \
    if (e_ != hipSuccess) {                                            \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                         \
    }                                                                  \
  } while (0)

__global__ void fill(uint16_t* p, size_t n, uint32_t seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 13;
    h *= 0x5bd1e995u;
    h ^= h >> 15;
    p[i] = (uint16_t)(0x3c00 + (h & 0x3ff) - 0x200);  // bf16 in roughly [-0.6, 0.6] x 2^-7 .. ordinary values
  }
}

int main(int argc, char** argv) {
  if (argc < 4) {
    fprintf(stderr, "usage: %s M N K [iters]\n", argv[0]);
    return 2;
  }
  const int M = atoi(argv[1]), N = atoi(argv[2]), K = atoi(argv[3]), iters = argc > 4 ? atoi(argv[4]) : 20,
            gm = argc > 5 ? atoi(argv[5]) : 4;
  if (N % 256 || K % 128 || M <= 0) {
    fprintf(stderr, "shape: N %% 256, K %% 128\n");
    return 2;
  }
  const size_t wn = (size_t)N * K;
  int nc = (int)((1ull << 30) / (wn * 2)) + 1;
  if (nc < 2) nc = 2;
  uint16_t *X, *Y;
  std::vector<uint16_t*> Ws(nc);
  CK(hipMalloc(&X, (size_t)M * K * 2));
  CK(hipMalloc(&Y, (size_t)M * N * 2));
  fill<<<1024, 256>>>(X, (size_t)M * K, 1);
  for (int i = 0; i < nc; ++i) {
    CK(hipMalloc(&Ws[i], wn * 2));
    fill<<<1024, 256>>>(Ws[i], wn, 7 + i);
  }
  CK(hipDeviceSynchronize());
  auto run = [&](int i) {
    const int rc = xot::launch_gemm_w4(X, K, Ws[i % nc], nullptr, nullptr, 0, Y, N, false, xot::EPI_NONE, nullptr, M,
                                       N, K, 1, gm, 0);
    if (rc) {
      fprintf(stderr, "launch rc %d\n", rc);
      exit(1);
    }
  };
  for (int i = 0; i < 3; ++i) run(i);
  CK(hipDeviceSynchronize());
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float best = 1e30f;
  for (int r = 0; r < 3; ++r) {
    CK(hipEventRecord(a, 0));
    for (int i = 0; i < iters; ++i) run(i);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    if (ms < best) best = ms;
  }
  const double us = best * 1e3 / iters;
#if W4_PROBE
  {  // average cycles per stage interval over blocks, waves and the 8 recorded stages of the last launch
    const int nblk = ((M + 255) / 256) * (N / 256) < 4096 ? ((M + 255) / 256) * (N / 256) : 4096;
    std::vector<unsigned long long> pr(4096 * 4 * 8 * 4);
    CK(hipMemcpyFromSymbol(pr.data(), HIP_SYMBOL(xot::w4_probe), pr.size() * 8));
    double acc[4] = {0, 0, 0, 0};
    long cnt = 0;
    for (int b = 0; b < nblk; ++b)
      for (int w = 0; w < 4; ++w)
        for (int s = 0; s < 8; ++s) {
          const unsigned long long* q = &pr[((b * 4 + w) * 8 + s) * 4];
          const unsigned long long* qn = &pr[((b * 4 + w) * 8 + ((s + 1) & 7)) * 4];
          if (s == 7 || qn[0] < q[3]) continue;  // intervals inside one launch only
          acc[0] += (double)(q[1] - q[0]);
          acc[1] += (double)(q[2] - q[1]);
          acc[2] += (double)(q[3] - q[2]);
          acc[3] += (double)(qn[0] - q[3]);
          ++cnt;
        }
    printf("{\"probe\": \"%s\", \"stages\": %ld, \"start_b1\": %.0f, \"b1_b2\": %.0f, \"b2_end\": %.0f, \"end_next\": %.0f}\n",
           VARIANT, cnt, acc[0] / cnt, acc[1] / cnt, acc[2] / cnt, acc[3] / cnt);
  }
#endif
  printf("{\"variant\": \"%s\", \"M\": %d, \"N\": %d, \"K\": %d, \"group_m\": %d, \"us\": %.1f, \"pflops\": %.3f}\n", VARIANT, M, N, K, gm, us,
         2.0 * M * N * K / us / 1e9);
  return 0;
}

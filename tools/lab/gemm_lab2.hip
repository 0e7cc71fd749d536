// Standalone GEMM lab (no torch): gemm_big_kernel variants on RANDOM bf16 operands with the weights rotated
// through >= 1 GB (HBM-cold per call, as in a forward pass), timed interleaved in one process.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/lab/gemm_lab2.hip -o tools/lab/gemm_lab2
//   ./tools/lab/gemm_lab2 M N K [variant]        variant -1 = all (interleaved rounds), else one (profiling)
#include "../../xotorch_support_jetson_amd/csrc/gemm_big.hip"
#include "../../xotorch_support_jetson_amd/csrc/gemm_sk.hip"
#include "gemm_w4.hip"
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace xot;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ void fill_rand(uint16_t* p, size_t n, uint32_t seed, float scale) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13; h *= 3266489917u; h ^= h >> 16;
    const float u = ((h & 0xffffff) / 16777216.0f) * 2.f - 1.f;  // uniform [-1, 1)
    p[i] = f2bf(u * scale);
  }
}

struct Ctx {
  const uint16_t* X; const uint16_t* W; uint16_t* Y; float* ws; int M, N, K; size_t wstride; int nc; int ldx;
};

typedef void (*LaunchFn)(const Ctx&, const uint16_t* W, hipStream_t);

template <int BN, int WM, int BK, int NBUF, int AUXA, int AUXB, bool PRIO, int PP, int EPI>
void launch_v(const Ctx& c, const uint16_t* W, hipStream_t st) {
  constexpr int WN = 8 / WM;
  constexpr int SMEM = big_smem<256, BN, BK, NBUF, PP>();
  auto k = gemm_big_kernel<256, BN, WM, WN, BK, NBUF, EPI, false, false, 0, 0, AUXA, AUXB, PRIO, PP>;
  static bool attr = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM) == hipSuccess;
  (void)attr;
  const int nwg = ((c.M + 255) / 256) * (c.N / BN);
  k<<<nwg, 512, SMEM, st>>>(c.X, c.ldx, W, nullptr, nullptr, 0, c.Y, EPI == EPI_SILU ? c.N / 2 : c.N, nullptr, c.M, c.N,
                            c.K, 1, nullptr, nullptr, 0L);
}

static float* g_part = nullptr;
static int* g_sync = nullptr;
template <int EPI>
void launch_sk(const Ctx& c, const uint16_t* W, hipStream_t st) {
  launch_gemm_sk(c.X, c.ldx, W, nullptr, nullptr, 0, c.Y, EPI == EPI_SILU ? c.N / 2 : c.N, false, EPI, g_part, g_sync, c.M,
                 c.N, c.K, 256, st);
}

template <int EPI, int DMA>
void launch_w4(const Ctx& c, const uint16_t* W, hipStream_t st) {
  auto k = gemm_w4_kernel<EPI, false, false, DMA>;
  static bool attr = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, w4::SMEM) == hipSuccess;
  (void)attr;
  const int nwg = ((c.M + 255) / 256) * (c.N / 256);
  k<<<nwg, 256, w4::SMEM, st>>>(c.X, c.ldx, W, nullptr, nullptr, 0, c.Y, EPI == EPI_SILU ? c.N / 2 : c.N, nullptr, c.M, c.N,
                                c.K, 1);
}

struct Variant { const char* name; LaunchFn fn; };

int main(int argc, char** argv) {
  const int M = atoi(argv[1]), N = atoi(argv[2]), K = atoi(argv[3]);
  const int only = argc > 4 ? atoi(argv[4]) : -1;
  const int epi = argc > 5 ? atoi(argv[5]) : EPI_SILU;
  const size_t wsz = (size_t)N * K;
  // weight copies rotated per call (HBM-cold); argv[6] = 1 keeps one copy (cache-resident when it fits), 0 = default
  const int nc_arg = argc > 6 ? atoi(argv[6]) : 0;  // <= 0: the rotating default
  const int nc = nc_arg > 0 ? nc_arg : (int)std::max<size_t>(2, (1ull << 30) / (wsz * 2) + 1);
  // argv[7] = X row padding in elements (row stride K + pad: rows at a non-power-of-two stride)
  const int ldx = K + (argc > 7 ? atoi(argv[7]) : 0);
  uint16_t *X, *W, *Y;
  CK(hipMalloc(&X, (size_t)M * ldx * 2));
  CK(hipMalloc(&W, wsz * 2 * nc));
  CK(hipMalloc(&Y, (size_t)M * N * 4));
  fill_rand<<<4096, 256>>>(X, (size_t)M * ldx, 17u, 1.0f);
  fill_rand<<<4096, 256>>>(W, wsz * nc, 91u, 0.02f);
  CK(hipDeviceSynchronize());
  Ctx c{X, W, Y, nullptr, M, N, K, wsz, nc, ldx};
  CK(hipMalloc(&g_part, gemm_sk_part_elems() * 4));
  CK(hipMalloc(&g_sync, 1 << 20));
  CK(hipMemset(g_sync, 0, 1 << 20));
  std::vector<Variant> vs;
  if (epi == EPI_SILU) {
    vs.push_back({"pp nt(B)     ", launch_v<256, 2, 64, 2, 0, 3, false, 1, EPI_SILU>});
    vs.push_back({"base 256     ", launch_v<256, 2, 64, 2, 0, 3, false, 0, EPI_SILU>});
    vs.push_back({"W 3-deep     ", launch_v<256, 2, 64, 2, 0, 3, false, 3, EPI_SILU>});
    if (N % 224 == 0) vs.push_back({"base 224     ", launch_v<224, 4, 64, 2, 0, 3, false, 0, EPI_SILU>});
    vs.push_back({"stream-K     ", launch_sk<EPI_SILU>});
  } else {
    vs.push_back({"pp nt(B)     ", launch_v<256, 2, 64, 2, 0, 3, false, 1, EPI_NONE>});
    vs.push_back({"base 256     ", launch_v<256, 2, 64, 2, 0, 3, false, 0, EPI_NONE>});
    vs.push_back({"W 3-deep     ", launch_v<256, 2, 64, 2, 0, 3, false, 3, EPI_NONE>});
    if (N % 224 == 0) vs.push_back({"base 224     ", launch_v<224, 4, 64, 2, 0, 3, false, 0, EPI_NONE>});
    vs.push_back({"stream-K     ", launch_sk<EPI_NONE>});
  }
  {  // every variant must produce the first variant's output (same tile math; k order identical)
    std::vector<uint16_t> ref((size_t)M * N), got((size_t)M * N);
    const size_t ny = (size_t)M * (epi == EPI_SILU ? N / 2 : N);
    for (size_t v = 0; v < vs.size(); ++v) {
      CK(hipMemset(Y, 0, (size_t)M * N * 4));
      vs[v].fn(c, W, 0);
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(v == 0 ? ref.data() : got.data(), Y, ny * 2, hipMemcpyDeviceToHost));
      if (v == 0) continue;
      double maxd = 0, maxr = 0;
      for (size_t i = 0; i < ny; ++i) {
        const float r = __builtin_bit_cast(float, (uint32_t)ref[i] << 16), g = __builtin_bit_cast(float, (uint32_t)got[i] << 16);
        maxd = std::max(maxd, (double)std::fabs(r - g));
        maxr = std::max(maxr, (double)std::fabs(r));
      }
      printf("check %s vs %s: max |diff| %.3g (max |ref| %.3g)\n", vs[v].name, vs[0].name, maxd, maxr);
    }
  }
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const double flop = 2.0 * M * N * K;
  const int rounds = only >= 0 ? 3 : 5, iters = 10;
  std::vector<std::vector<float>> t(vs.size());
  int call = 0;
  for (int r = 0; r < rounds; ++r)
    for (size_t v = 0; v < vs.size(); ++v) {
      if (only >= 0 && (int)v != only) continue;
      for (int w = 0; w < 2; ++w) vs[v].fn(c, W + (size_t)((call++) % nc) * wsz, 0);
      CK(hipEventRecord(a));
      for (int i = 0; i < iters; ++i) vs[v].fn(c, W + (size_t)((call++) % nc) * wsz, 0);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      t[v].push_back(ms * 1e3f / iters);
    }
  for (size_t v = 0; v < vs.size(); ++v) {
    if (t[v].empty()) continue;
    std::sort(t[v].begin(), t[v].end());
    printf("M=%d N=%d K=%d %s median %8.1f us (%6.0f TF/s)  min %8.1f us\n", M, N, K, vs[v].name,
           t[v][t[v].size() / 2], flop / t[v][t[v].size() / 2] / 1e6, t[v][0]);
  }
  return 0;
}

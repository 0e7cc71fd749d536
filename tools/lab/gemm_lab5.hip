// GEMM lab 5: the two-phase ping-pong schedule (gemm_big PP 2, tile code 2256) against the four-phase one (PP 1)
// and the base schedule, on the production kernel, HBM-cold random operands (harness of lab 3).  Variants
// measured on the way and not kept (logs in profiles/r4/pp2/): every phase barrier but the refill one dropped
// (racy by design, timing only: not faster), the refill moved behind the phase barrier, and only the A rows still
// being read moved there (both slower than four phases).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/lab/gemm_lab5.hip -o tools/lab/gemm_lab5
//   ./tools/lab/gemm_lab5 M N K S
#include "../../xotorch_support_jetson_amd/csrc/gemm_big.hip"
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

struct Ctx { const uint16_t* X; uint16_t* Y; float* ws; int M, N, K, S, epi; };
typedef void (*LaunchFn)(const Ctx&, const uint16_t* W, hipStream_t);

template <int BM, int BN, int WM, int BK, int NBUF, int PP, int AUXB, int EPI>
void launch_v(const Ctx& c, const uint16_t* W, hipStream_t st) {
  constexpr int WN = 8 / WM;
  constexpr int SMEM = big_smem<BM, BN, BK, NBUF>();
  static_assert(SMEM <= 160 * 1024, "LDS");
  const int nwg = ((c.M + BM - 1) / BM) * (c.N / BN) * c.S;
  if (c.S == 1) {
    auto k = gemm_big_kernel<BM, BN, WM, WN, BK, NBUF, EPI, false, false, 0, 0, AUXB, PP>;
    static bool attr = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM) == hipSuccess;
    (void)attr;
    k<<<nwg, 512, SMEM, st>>>(c.X, c.K, W, nullptr, nullptr, 0, c.Y, EPI == EPI_SILU ? c.N / 2 : c.N, nullptr, c.M, c.N,
                              c.K, 1, nullptr, nullptr, 0L, 4);
  } else {
    auto k = gemm_big_kernel<BM, BN, WM, WN, BK, NBUF, EPI_NONE, false, true, 0, 0, AUXB, PP>;
    static bool attr = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM) == hipSuccess;
    (void)attr;
    k<<<nwg, 512, SMEM, st>>>(c.X, c.K, W, nullptr, nullptr, 0, c.Y, c.N, c.ws, c.M, c.N, c.K, c.S, nullptr, nullptr, 0L, 4);
  }
}

static float* g_part = nullptr;
static int* g_sync = nullptr;

struct Variant { const char* name; LaunchFn fn; };

template <int EPI>
std::vector<Variant> variants(int S) {
  std::vector<Variant> vs;
  vs.push_back({"pp   256x256 BK64   ", launch_v<256, 256, 2, 64, 2, 1, 3, EPI>});
  vs.push_back({"pp2  two phases     ", launch_v<256, 256, 2, 64, 2, 2, 3, EPI>});
  vs.push_back({"base 256x256 BK64   ", launch_v<256, 256, 2, 64, 2, 0, 3, EPI>});
  return vs;
}

int main(int argc, char** argv) {
  if (argc < 5) { printf("usage: M N K S [variant] [epi]\n"); return 1; }
  const int M = atoi(argv[1]), N = atoi(argv[2]), K = atoi(argv[3]), S = atoi(argv[4]);
  const int only = argc > 5 ? atoi(argv[5]) : -1;
  const int epi = argc > 6 ? atoi(argv[6]) : (S == 1 ? EPI_SILU : EPI_NONE);
  if (M > 8192 || N % 256 || K % 128 || S < 1 || (S > 1 && epi != EPI_NONE)) { printf("bad shape\n"); return 1; }
  const size_t wsz = (size_t)N * K;
  const int nc = (int)std::max<size_t>(2, (1ull << 30) / (wsz * 2) + 1);  // weight copies rotated: HBM-cold calls
  uint16_t *X, *W, *Y;
  float* ws = nullptr;
  CK(hipMalloc(&X, (size_t)M * K * 2));
  CK(hipMalloc(&W, wsz * 2 * nc));
  CK(hipMalloc(&Y, (size_t)M * N * 4));
  if (S > 1) CK(hipMalloc(&ws, (size_t)S * M * N * 4));
  fill_rand<<<4096, 256>>>(X, (size_t)M * K, 17u, 1.0f);
  fill_rand<<<4096, 256>>>(W, wsz * nc, 91u, 0.02f);
  CK(hipDeviceSynchronize());
  CK(hipMalloc(&g_part, 4096));
  CK(hipMalloc(&g_sync, 1 << 20));
  CK(hipMemset(g_sync, 0, 1 << 20));
  Ctx c{X, Y, ws, M, N, K, S, epi};
  std::vector<Variant> vs = epi == EPI_SILU ? variants<EPI_SILU>(S) : variants<EPI_NONE>(S);
  {  // every variant must give the first variant's output (bf16 out, or the summed fp32 slabs)
    const size_t ny = S > 1 ? (size_t)M * N : (size_t)M * (epi == EPI_SILU ? N / 2 : N);
    std::vector<float> ref(ny), got(ny);
    std::vector<uint16_t> h16(ny);
    std::vector<float> h32((size_t)S * M * N);
    for (size_t v = 0; v < vs.size(); ++v) {
      if (only >= 0 && v != 0 && (int)v != only) continue;
      CK(hipMemset(Y, 0, (size_t)M * N * 4));
      if (ws) CK(hipMemset(ws, 0, (size_t)S * M * N * 4));
      vs[v].fn(c, W, 0);
      CK(hipDeviceSynchronize());
      std::vector<float>& dst = v == 0 ? ref : got;
      if (S > 1) {
        CK(hipMemcpy(h32.data(), ws, h32.size() * 4, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < ny; ++i) { float a = 0; for (int s = 0; s < S; ++s) a += h32[(size_t)s * ny + i]; dst[i] = a; }
      } else {
        CK(hipMemcpy(h16.data(), Y, ny * 2, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < ny; ++i) dst[i] = __builtin_bit_cast(float, (uint32_t)h16[i] << 16);
      }
      if (v == 0) continue;
      double maxd = 0, maxr = 0;
      for (size_t i = 0; i < ny; ++i) { maxd = std::max(maxd, (double)std::fabs(ref[i] - got[i])); maxr = std::max(maxr, (double)std::fabs(ref[i])); }
      printf("check %s vs %s: max |diff| %.3g (max |ref| %.3g)%s\n", vs[v].name, vs[0].name, maxd, maxr,
             maxd > 0.02 * maxr ? "  MISMATCH" : "");
      // (diagnostic variants may race: report only)
    }
  }
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const double flop = 2.0 * M * N * K;
  const int rounds = only >= 0 ? (getenv("LAB_ROUNDS") ? atoi(getenv("LAB_ROUNDS")) : 3) : 5, iters = 10;  // LAB_ROUNDS: long runs (power, PMC)
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
    printf("M=%d N=%d K=%d S=%d %s median %8.1f us (%6.0f TF/s)  min %8.1f us\n", M, N, K, S, vs[v].name,
           t[v][t[v].size() / 2], flop / t[v][t[v].size() / 2] / 1e6, t[v][0]);
  }
  return 0;
}

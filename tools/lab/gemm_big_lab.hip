// Standalone ablation bench of gemm_big_kernel (no torch): which part of the k loop bounds it, per
// tile / stage configuration.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/lab/gemm_big_lab.hip -o tools/lab/gemm_big_lab
//   ./tools/lab/gemm_big_lab M N K S
#include "../../xotorch_support_jetson_amd/csrc/gemm_big.hip"
#include <algorithm>
#include <cstdio>
#include <cstdlib>

using namespace xot;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

static int g_ldx_pad = 0;  // extra elements per X row (L2 channel spread experiment)

template <int BN, int BK, int NBUF, int ABL, int AA = 0, int AB = 0, bool PRIO = false, bool PP = false>
float run(const uint16_t* X, const uint16_t* W, uint16_t* Y, float* ws, int M, int N, int K, int S, size_t wstride,
          int ncopies) {
  const int ldx = K + g_ldx_pad;
  constexpr int WM = BN == 256 ? 2 : 4, WN = 8 / WM;
  constexpr int SMEM = NBUF * (256 + BN) * BK * 2;
  const int nwg = ((M + 255) / 256) * (N / BN) * S;
  auto k1 = gemm_big_kernel<256, BN, WM, WN, BK, NBUF, EPI_NONE, false, false, 0, ABL, AA, AB, PRIO, PP>;
  auto k2 = gemm_big_kernel<256, BN, WM, WN, BK, NBUF, EPI_NONE, false, true, 0, ABL, AA, AB, PRIO, PP>;
  CK(hipFuncSetAttribute((const void*)k1, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM));
  CK(hipFuncSetAttribute((const void*)k2, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float best = 1e30f;
  for (int r = 0; r < 12; ++r) {
    const uint16_t* Wc = W + (size_t)(r % ncopies) * wstride;
    CK(hipEventRecord(a));
    if (S == 1) k1<<<nwg, 512, SMEM>>>(X, ldx, Wc, nullptr, nullptr, 0, Y, N, nullptr, M, N, K, 1, nullptr, nullptr, 0L);
    else k2<<<nwg, 512, SMEM>>>(X, ldx, Wc, nullptr, nullptr, 0, Y, N, ws, M, N, K, S, nullptr, nullptr, 0L);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    if (r >= 2 && ms < best) best = ms;
  }
  return best * 1e3f;
}

template <int BN, int BK, int NBUF, int AB = 3>
void sweep(const uint16_t* X, const uint16_t* W, uint16_t* Y, float* ws, int M, int N, int K, int S, size_t wsz,
           int nc, bool abl) {
  if (N % BN) return;
  const double flop = 2.0 * M * N * K;
  const char* names[4] = {"full", "no-mfma", "no-loads", "serial"};
  float us[4] = {run<BN, BK, NBUF, 0, 0, AB>(X, W, Y, ws, M, N, K, S, wsz, nc), 0, 0, 0};
  if (abl) {
    us[1] = run<BN, BK, NBUF, 1, 0, AB>(X, W, Y, ws, M, N, K, S, wsz, nc);
    us[2] = run<BN, BK, NBUF, 2, 0, AB>(X, W, Y, ws, M, N, K, S, wsz, nc);
    us[3] = run<BN, BK, NBUF, 3, 0, AB>(X, W, Y, ws, M, N, K, S, wsz, nc);
  }
  for (int a = 0; a < (abl ? 4 : 1); ++a)
    printf("M=%d N=%d K=%d S=%d BN=%d BK=%d NBUF=%d %-9s %8.1f us %7.1f TF/s\n", M, N, K, S, BN, BK, NBUF, names[a],
           us[a], flop / us[a] / 1e6);
  fflush(stdout);
}

int main(int argc, char** argv) {
  const int M = atoi(argv[1]), N = atoi(argv[2]), K = atoi(argv[3]), S = atoi(argv[4]);
  const bool abl = argc > 5 && atoi(argv[5]);
  const int only = argc > 6 ? atoi(argv[6]) : -1;  // run one configuration (profiling)
  const size_t wsz = (size_t)N * K;
  const int nc = (int)std::max<size_t>(2, (1ull << 30) / (wsz * 2) + 1);
  uint16_t *X, *W, *Y;
  float* ws;
  CK(hipMalloc(&X, (size_t)M * (K + 1024) * 2));
  CK(hipMalloc(&W, wsz * 2 * nc));
  CK(hipMalloc(&Y, (size_t)M * N * 4));
  CK(hipMalloc(&ws, (size_t)S * M * N * 4));
  CK(hipMemset(X, 0x3c, (size_t)M * (K + 1024) * 2));
  CK(hipMemset(W, 0x3c, wsz * 2 * nc));
  if (only < 0 || only == 0) sweep<256, 64, 2>(X, W, Y, ws, M, N, K, S, wsz, nc, abl);
  if (only < 0 || only == 1) sweep<256, 32, 4>(X, W, Y, ws, M, N, K, S, wsz, nc, abl);
  if (only < 0 || only == 2) sweep<256, 32, 3>(X, W, Y, ws, M, N, K, S, wsz, nc, abl);
  if (only < 0 || only == 3) sweep<128, 64, 3>(X, W, Y, ws, M, N, K, S, wsz, nc, abl);
  if (only < 0 || only == 4) sweep<128, 32, 4>(X, W, Y, ws, M, N, K, S, wsz, nc, abl);
  if (only == 6) {  // ping-pong schedule vs the one-barrier-per-stage loop
    const double flop = 2.0 * M * N * K;
    for (int rep = 0; rep < 2; ++rep) {
      const float a = run<256, 64, 2, 0, 0, 3>(X, W, Y, ws, M, N, K, S, wsz, nc);
      const float b = run<256, 64, 2, 0, 0, 3, false, true>(X, W, Y, ws, M, N, K, S, wsz, nc);
      printf("M=%d N=%d K=%d S=%d base %.1f us (%.0f TF/s)  pp %.1f us (%.0f TF/s)\n", M, N, K, S, a, flop / a / 1e6, b,
             flop / b / 1e6);
    }
  }
  if (only == 7) {  // X row stride padding
    const double flop = 2.0 * M * N * K;
    for (int pad : {0, 64, 128, 512, 0}) {
      g_ldx_pad = pad;
      const float a = run<256, 64, 2, 0, 0, 3>(X, W, Y, ws, M, N, K, S, wsz, nc);
      const float b = run<256, 64, 2, 1, 0, 3>(X, W, Y, ws, M, N, K, S, wsz, nc);
      printf("ldx pad %4d: full %.1f us (%.0f TF/s)  no-mfma %.1f us\n", pad, a, flop / a / 1e6, b);
    }
    g_ldx_pad = 0;
  }
  if (only == 8) {  // s_setprio around the MFMA clusters
    const double flop = 2.0 * M * N * K;
    for (int rep = 0; rep < 2; ++rep) {
      float a = run<256, 64, 2, 0, 0, 3, false>(X, W, Y, ws, M, N, K, S, wsz, nc);
      float b = run<256, 64, 2, 0, 0, 3, true>(X, W, Y, ws, M, N, K, S, wsz, nc);
      float c = run<256, 64, 2, 2, 0, 3, false>(X, W, Y, ws, M, N, K, S, wsz, nc);
      float d = run<256, 64, 2, 2, 0, 3, true>(X, W, Y, ws, M, N, K, S, wsz, nc);
      printf("prio off %.1f us (%.0f TF/s)  on %.1f us (%.0f TF/s) | no-loads off %.1f on %.1f\n", a, flop / a / 1e6, b,
             flop / b / 1e6, c, d);
    }
  }
  if (only == 9) {  // cache-policy bits on the 256x256x64 tile
    const double flop = 2.0 * M * N * K;
#define AUXRUN(AA, AB) printf("aux A=%d B=%d: %8.1f us %7.1f TF/s\n", AA, AB, run<256, 64, 2, 0, AA, AB>(X, W, Y, ws, M, N, K, S, wsz, nc), flop / run<256, 64, 2, 0, AA, AB>(X, W, Y, ws, M, N, K, S, wsz, nc) / 1e6)
    AUXRUN(0, 0); AUXRUN(0, 2); AUXRUN(2, 0); AUXRUN(2, 2); AUXRUN(1, 1); AUXRUN(0, 1); AUXRUN(0, 16); AUXRUN(0, 17);
    AUXRUN(0, 3); AUXRUN(16, 16);
  }
  return 0;
}

// Layout kernels for the training GEMMs: the pre-shuffled MFMA operand layout of the gemm_big / stream
// kernels (16-row x 128-k tiles, [N/16][K/128][4][lane][8], lane = 16 g + c holds row c, k 8 g .. 8 g + 7 of
// each 32-deep step; ops/weights_layout.py:shuffle_for_stream), built on the device each optimizer step /
// micro-batch instead of once at load:
//   shuffle    dst = shuffle(src)        src [R, C] row-major (row stride ld)          -> the W operand of y = x W^T
//   shuffle_t  dst = shuffle(src^T)      src [R, C] -> [C, R] shuffled                -> W^T (dX = dY W), X^T (dW)
//   transpose  dst = src^T row-major     src [R, C] -> [C, R]                          -> dY^T (the A operand of dW)
// shuffle is a pure 16-byte permutation (one chunk per thread, coalesced writes); the two transposing kernels
// stage a 128 (R) x 64 (C) tile through LDS, transposed on the way in (stage_tile_t).
#include "common.h"
#include "kernels.h"

namespace xot {

__global__ __launch_bounds__(256) void shuffle_kernel(const uint16_t* __restrict__ src, long ld,
                                                      uint16_t* __restrict__ dst, int R, int C) {
  const long chunks = (long)R * C / 8;
  const int KC = C / 128;
  for (long q = (long)blockIdx.x * 256 + threadIdx.x; q < chunks; q += (long)gridDim.x * 256) {
    const int lane = (int)(q & 63);
    const long t = q >> 6;  // ((nt * KC + kc) * 4 + s)
    const int s = (int)(t & 3);
    const long u = t >> 2;
    const int kc = (int)(u % KC);
    const long nt = u / KC;
    const long row = nt * 16 + (lane & 15);
    const int col = kc * 128 + s * 32 + (lane >> 4) * 8;
    st16(dst + q * 8, ld16(src + row * ld + col));
  }
}

// tile: TR = 128 rows of src (= k of the transposed matrix), TC = 64 columns (= its rows), staged TRANSPOSED in
// LDS as ldt[c][r] with a 16-B-aligned pitch: two src rows' 16-B chunks are interleaved into 32-bit words (8
// ds_write_b32 per row pair instead of 16 ds_write_b16), and every output chunk -- 8 consecutive r of one c --
// is one ds_read_b128 (the first version wrote and read 2-byte LDS words: 64 LDS instructions per thread, ~3.3
// TB/s on the training step's dY^T / shuffle(X^T)).
constexpr int TR = 128, TC = 64, TRP = TR + 8;  // LDS pitch of a transposed row (272 B)

__device__ __forceinline__ void stage_tile_t(const uint16_t* __restrict__ src, long ld, int r0, int c0,
                                             uint16_t* ldt) {
#pragma unroll
  for (int i = 0; i < TR * TC / 16 / 256; ++i) {  // 2 row pairs x 8 columns per thread
    const int q = i * 256 + threadIdx.x;
    const int pr = q >> 3, c8 = (q & 7) * 8;
    const s16x8 a = ld16(src + (long)(r0 + 2 * pr) * ld + c0 + c8);
    const s16x8 b = ld16(src + (long)(r0 + 2 * pr + 1) * ld + c0 + c8);
#pragma unroll
    for (int e = 0; e < 8; ++e)
      *reinterpret_cast<uint32_t*>(ldt + (c8 + e) * TRP + 2 * pr) =
          (uint32_t)(uint16_t)a[e] | ((uint32_t)(uint16_t)b[e] << 16);
  }
}

__global__ __launch_bounds__(256) void shuffle_t_kernel(const uint16_t* __restrict__ src, long ld,
                                                        uint16_t* __restrict__ dst, int R, int C) {
  __shared__ __attribute__((aligned(16))) uint16_t ldt[TC * TRP];
  const int r0 = blockIdx.x * TR, c0 = blockIdx.y * TC;  // a 128-deep k chunk (kc) x 4 row groups (nt)
  stage_tile_t(src, ld, r0, c0, ldt);
  __syncthreads();
  const int KC = R / 128, kc = r0 / 128;
#pragma unroll
  for (int i = 0; i < 4; ++i) {  // 4 nt x 4 s x 64 lanes = 1024 chunks of 8
    const int q = i * 256 + threadIdx.x;
    const int lane = q & 63, s = (q >> 6) & 3, ntl = q >> 8;
    const int n = ntl * 16 + (lane & 15);        // row of src^T inside the tile (= src column)
    const int k = s * 32 + (lane >> 4) * 8;      // first k (= src row) inside the tile
    const long nt = c0 / 16 + ntl;
    st16(dst + (((nt * KC + kc) * 4 + s) * 64 + lane) * 8, ld16(ldt + n * TRP + k));
  }
}

__global__ __launch_bounds__(256) void transpose_kernel(const uint16_t* __restrict__ src, long ld,
                                                        uint16_t* __restrict__ dst, int R, int C) {
  __shared__ __attribute__((aligned(16))) uint16_t ldt[TC * TRP];
  const int r0 = blockIdx.x * TR, c0 = blockIdx.y * TC;
  stage_tile_t(src, ld, r0, c0, ldt);
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 4; ++i) {  // dst rows c0 .. c0+63, each 128 wide = 16 chunks of 8
    const int q = i * 256 + threadIdx.x;
    const int c = q >> 4, r8 = (q & 15) * 8;
    st16(dst + (long)(c0 + c) * R + r0 + r8, ld16(ldt + c * TRP + r8));
  }
}


int launch_shuffle(const uint16_t* src, long ld, uint16_t* dst, int R, int C, hipStream_t s) {
  if (R % 16 || C % 128) return -1;
  const long chunks = (long)R * C / 8;
  if (chunks == 0) return 0;
  const int blocks = (int)std::min<long>((chunks + 255) / 256, 8192);
  shuffle_kernel<<<blocks, 256, 0, s>>>(src, ld, dst, R, C);
  return 0;
}

int launch_shuffle_t(const uint16_t* src, long ld, uint16_t* dst, int R, int C, hipStream_t s) {
  if (R % TR || C % TC) return -1;
  if (R == 0 || C == 0) return 0;
  shuffle_t_kernel<<<dim3(R / TR, C / TC), 256, 0, s>>>(src, ld, dst, R, C);
  return 0;
}

int launch_transpose(const uint16_t* src, long ld, uint16_t* dst, int R, int C, hipStream_t s) {
  if (R % TR || C % TC) return -1;
  if (R == 0 || C == 0) return 0;
  transpose_kernel<<<dim3(R / TR, C / TC), 256, 0, s>>>(src, ld, dst, R, C);
  return 0;
}

}  // namespace xot

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


// ---- v2 (round 6): 128 x 128 tiles staged row-major (16-B LDS writes, 144-element pitch = 8 dwords mod 64) and read
// back TRANSPOSED with ds_read_b64_tr_b16: a 16-lane group's two reads return, lane c, src column c of a 16-column
// block at 8 consecutive src rows -- exactly one 8-element output chunk, so every store is 16 B and a wave's four
// groups write 64 B (transpose) / 1 KB (shuffle_t) contiguous.  Column tiles are the fastest grid dimension: the
// blocks in flight together read adjacent 256-B segments of the same 128 src rows (the v1 grid walked down the
// rows of one 128-B column strip, ~1.1 TB/s on the training step's dY^T).
typedef __attribute__((address_space(3))) s16x4* lds_s16x4_t;
constexpr int T2 = 128, T2P = T2 + 16;

__device__ __forceinline__ void stage_tile_rows(const uint16_t* __restrict__ src, long ld, int r0, int c0,
                                                uint16_t* lt) {
#pragma unroll
  for (int i = 0; i < T2 * T2 / 8 / 256; ++i) {  // 2048 chunks of 8, 16 per row
    const int q = i * 256 + threadIdx.x;
    const int r = q >> 4, c8 = (q & 15) * 8;
    *reinterpret_cast<s16x8*>(lt + r * T2P + c8) = ld16(src + (long)(r0 + r) * ld + c0 + c8);
  }
}

// 8 consecutive tile rows rr .. rr+7 of tile column cc + (lane c of the 16-lane group), from the row-major LDS tile
__device__ __forceinline__ s16x8 tr_chunk(const uint16_t* lt, int rr, int cc, int c) {
  const uint16_t* p = lt + (rr + (c >> 2)) * T2P + cc + 4 * (c & 3);
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t)(p));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t)(p + 4 * T2P));
  return s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

__global__ __launch_bounds__(256) void transpose2_kernel(const uint16_t* __restrict__ src, long ld,
                                                         uint16_t* __restrict__ dst, int R, int C) {
  __shared__ __attribute__((aligned(16))) uint16_t lt[T2 * T2P];
  const int c0 = blockIdx.x * T2, r0 = blockIdx.y * T2;
  stage_tile_rows(src, ld, r0, c0, lt);
  __syncthreads();
  const int lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15, wave = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < 8; ++i) {  // 128 groups = 8 column blocks x 16 row blocks of 8
    const int G = i * 16 + wave * 4 + g, rb = G & 15, cb = G >> 4;
    st16(dst + (long)(c0 + cb * 16 + c) * R + r0 + rb * 8, tr_chunk(lt, rb * 8, cb * 16, c));
  }
}

__global__ __launch_bounds__(256) void shuffle_t2_kernel(const uint16_t* __restrict__ src, long ld,
                                                         uint16_t* __restrict__ dst, int R, int C) {
  __shared__ __attribute__((aligned(16))) uint16_t lt[T2 * T2P];
  const int c0 = blockIdx.x * T2, r0 = blockIdx.y * T2;  // 8 row groups (nt) x one 128-deep k chunk (kc)
  stage_tile_rows(src, ld, r0, c0, lt);
  __syncthreads();
  const int lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15, wave = threadIdx.x >> 6;
  const int KC = R / 128, kc = r0 / 128;
#pragma unroll
  for (int i = 0; i < 8; ++i) {  // 128 groups = 8 nt x 4 k-steps (s) x 4 lane groups (g')
    const int G = i * 16 + wave * 4 + g, gp = G & 3, st = (G >> 2) & 3, ntl = G >> 4;
    const long nt = c0 / 16 + ntl;
    st16(dst + (((nt * KC + kc) * 4 + st) * 64 + 16 * gp + c) * 8, tr_chunk(lt, st * 32 + gp * 8, ntl * 16, c));
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

int launch_shuffle_t(const uint16_t* src, long ld, uint16_t* dst, int R, int C, hipStream_t s, int variant) {
  if (variant == 2 && R % T2 == 0 && C % T2 == 0) {
    if (R == 0 || C == 0) return 0;
    shuffle_t2_kernel<<<dim3(C / T2, R / T2), 256, 0, s>>>(src, ld, dst, R, C);
    return 0;
  }
  if (R % TR || C % TC) return -1;
  if (R == 0 || C == 0) return 0;
  shuffle_t_kernel<<<dim3(R / TR, C / TC), 256, 0, s>>>(src, ld, dst, R, C);
  return 0;
}

int launch_transpose(const uint16_t* src, long ld, uint16_t* dst, int R, int C, hipStream_t s, int variant) {
  if (variant == 2 && R % T2 == 0 && C % T2 == 0) {
    if (R == 0 || C == 0) return 0;
    transpose2_kernel<<<dim3(C / T2, R / T2), 256, 0, s>>>(src, ld, dst, R, C);
    return 0;
  }
  if (R % TR || C % TC) return -1;
  if (R == 0 || C == 0) return 0;
  transpose_kernel<<<dim3(R / TR, C / TC), 256, 0, s>>>(src, ld, dst, R, C);
  return 0;
}

}  // namespace xot

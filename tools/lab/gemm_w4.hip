// LAB ONLY -- measured slower than gemm_big's ping-pong tile (profiles/r3/lab_gemm_w4_vs_pp.log): hipcc keeps
// the 256 accumulators in AGPRs but runs out of the 256 arch VGPRs and shuffles through AGPRs in the k loop.
// Large-M projection GEMM, four-wave variant:  Y[M,N] = X[M,K] . W[N,K]^T on the pre-shuffled weight layout
//
// Same 256 x 256 x 64 workgroup tile as gemm_big, but 4 waves (one per SIMD, 256 threads) as 2 x 2, each
// owning a 128 x 128 output block = 8 x 8 tiles of v_mfma_f32_16x16x32_bf16 (256 accumulator registers of
// the 512 a lone wave may use).  Per 32-deep k step a wave reads 8 A + 8 B fragments from LDS for 64 MFMAs
// (4 MFMAs per fragment read; the 8-wave 128 x 64 blocks of gemm_big get 2.7), so LDS read traffic per FLOP
// falls by a third.  Operands are staged through registers: every thread loads 8 X and 8 W 16-byte chunks
// of the next k stage with plain global loads (the compiler's own vmcnt tracking, no LDS-DMA issue cost on a
// wave that is alone on its SIMD) and writes them to the other LDS buffer interleaved with the second k
// step's MFMAs; one barrier per 64-deep stage.
//   * X image: [256 rows][64 k], 16-B slot XOR-swizzled by (row >> 1) & 7 at the write (conflict-free
//     ds_read_b128 fragment groups); W image: the shuffled layout's 1 KB fragment blocks copied verbatim
//   * XCD-aware bijective tile order, split-K fp32 slabs, epilogues none / residual / SiLU(gate) * up
//
// Reference parity: the q/k/v/o and w1/w2/w3 projections of xotorch/inference/torch/models/
// general_mha.py:77-120 and llm_utils.py:513-522 (torchtune nn.Linear).
// (research kernel: included by gemm_lab2.hip after the production headers; not built into the library)

namespace xot {

namespace w4 {
constexpr int BM = 256, BN = 256, BK = 64, KS = BK / 32;
constexpr int MT = 8, NT = 8;                     // 16 x 16 tiles per wave (128 x 128)
constexpr int A_ELEMS = BM * BK, STAGE = (BM + BN) * BK;
constexpr int CH = 8;                             // 16-B chunks per thread per operand per stage
constexpr int SMEM = 2 * STAGE * 2;               // 128 KB
}  // namespace w4

// DMA = 0: both operands staged through registers; 1: W by LDS-DMA, X through registers; 2: both by LDS-DMA
template <int EPI, bool OUT_F32, bool SPLIT, int DMA = 0>
__global__ __launch_bounds__(256, 1) void gemm_w4_kernel(const uint16_t* __restrict__ X, int ldx,
                                                         const uint16_t* __restrict__ W,
                                                         const uint16_t* __restrict__ bias,
                                                         const uint16_t* R, int ldr, void* Yv, int ldy,
                                                         float* __restrict__ ws, int M, int N, int K, int S) {
  using namespace w4;
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c = lane & 15;
  const int wm = wave >> 1, wn = wave & 1;

  // ---- tile (bijective XCD remap, then split-major / column / row order, as gemm_big)
  const int mtiles = (M + BM - 1) / BM, ntiles = N / BN;
  const int nwg = mtiles * ntiles * S;
  int b = blockIdx.x;
  {
    const int xcd = b & 7, q = nwg >> 3, r = nwg & 7;
    b = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
  }
  const int mt = b % mtiles, nt = (b / mtiles) % ntiles, split = b / (mtiles * ntiles);
  const int m0 = mt * BM, n0 = nt * BN;
  const int T_all = K / BK;
  const int t_beg = (int)((long)split * T_all / S), t_end = (int)((long)(split + 1) * T_all / S);
  const int T = t_end - t_beg;

  auto aswz = [](int row) -> int { return (row >> 1) & 7; };
  // staging: chunk q = tid + 256 i.  X: row q / 8, logical slot q % 8 -> LDS slot (q % 8) ^ aswz(row).
  // W: 1 KB block q / 64 (16-column group (q / 64) / 2, k block (q / 64) % 2), lane q % 64.
  // X chunk i of thread tid: row (tid >> 3) + 32 i, slot tid & 7; the swizzle (row >> 1) & 7 = (tid >> 4) & 7
  // is the same for every i, so the LDS destinations are one offset plus constants
  const uint16_t* xsrc[CH];
#pragma unroll
  for (int i = 0; i < CH; ++i) {
    const int row = (tid >> 3) + 32 * i;
    xsrc[i] = X + (size_t)min(m0 + row, M - 1) * ldx + (tid & 7) * 8;  // rows past M: valid memory, masked
  }
  const int xdst0 = (tid >> 3) * BK + (((tid & 7) ^ ((tid >> 4) & 7)) * 8);
  // W chunk i: 1 KB block (tid >> 6) + 4 i = 16-column group 2 i + (tid >> 7), k block (tid >> 6) & 1
  const size_t kchunks = K / 128;
  const uint16_t* wsrc = W + ((size_t)(n0 >> 4) + (tid >> 7)) * kchunks * 2048 + ((tid >> 6) & 1) * 512 + (tid & 63) * 8;
  const size_t wstep = 2 * kchunks * 2048;  // two 16-column groups
  s16x8 sx[CH], sw[CH];
  auto gload = [&](int t) {
    const int k0 = (t_beg + t) * BK;
    const uint16_t* wk = wsrc + (size_t)(k0 >> 7) * 2048 + ((k0 & 127) >> 5) * 512;
#pragma unroll
    for (int i = 0; i < CH; ++i) sx[i] = ld16(xsrc[i] + k0);
    if constexpr (DMA == 0) {
#pragma unroll
      for (int i = 0; i < CH; ++i) sw[i] = __builtin_nontemporal_load(reinterpret_cast<const s16x8*>(wk + i * wstep));
    }
  };
  auto swrite = [&](int buf, int i) {  // chunk i of the register-staged operands -> LDS buffer buf
    uint16_t* As = smem + buf * STAGE;
    if constexpr (DMA < 2) st16(As + xdst0 + 32 * i * BK, sx[i]);
    if constexpr (DMA == 0) st16(As + A_ELEMS + (tid + 256 * i) * 8, sw[i]);
  };
  // LDS-DMA: instruction i of wave w copies X rows 8 (8 w + i) .. +8 (slot swizzle on the per-lane source
  // address) and W block 8 w + i (16-column group (8 w + i) / 2, k block i & 1) verbatim
  const uint16_t* dxsrc[CH];
#pragma unroll
  for (int i = 0; i < CH; ++i) {
    const int row = 8 * (8 * wave + i) + lane / 8;
    dxsrc[i] = X + (size_t)min(m0 + row, M - 1) * ldx + (((lane % 8) ^ aswz(row)) * 8);
  }
  const uint16_t* dwsrc = W + ((size_t)(n0 >> 4) + 4 * wave) * kchunks * 2048 + lane * 8;
  auto issue = [&](int t, int buf) {
    uint16_t* As = smem + buf * STAGE;
    const int k0 = (t_beg + t) * BK;
    const size_t woff = (size_t)(k0 >> 7) * 2048 + ((k0 & 127) >> 5) * 512;
    if constexpr (DMA == 2) {
#pragma unroll
      for (int i = 0; i < CH; ++i) glds16<0>(dxsrc[i] + k0, As + (8 * wave + i) * 512);
    }
#pragma unroll
    for (int i = 0; i < CH; ++i)
      glds16<3>(dwsrc + (size_t)(i >> 1) * kchunks * 2048 + (i & 1) * 512 + woff, As + A_ELEMS + (8 * wave + i) * 512);
  };

  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment offsets: A rows wm * 128 + 16 i + c (the swizzle (c >> 1) & 7 is the same for every i);
  // B: 16-column group wn * 8 + j, k block s2
  int aoff0[KS];
#pragma unroll
  for (int s2 = 0; s2 < KS; ++s2) {
    const int row = wm * 128 + c;
    aoff0[s2] = row * BK + (((4 * s2 + g) ^ aswz(row)) * 8);
  }
  const int boff = A_ELEMS + (wn * NT) * KS * 512 + lane * 8;

  // one 64-deep stage from LDS buffer buf; the staged chunks of the next stage go to the other buffer between
  // the MFMA rows of the second k step.  The loop is uniform: the last stage also writes (the other buffer
  // is never read again) and a load past the end re-reads the last stage, so no iteration has a branch.
  auto compute = [&](int buf) {
    const uint16_t* As = smem + buf * STAGE;
#pragma unroll
    for (int s2 = 0; s2 < KS; ++s2) {
      s16x8 bf[NT];
#pragma unroll
      for (int j = 0; j < NT; ++j) bf[j] = ld16(As + boff + (j * KS + s2) * 512);
      s16x8 af[2];
      af[0] = ld16(As + aoff0[s2]);
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        if (i + 1 < MT) af[(i + 1) & 1] = ld16(As + aoff0[s2] + (i + 1) * 16 * BK);
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = mfma16(af[i & 1], bf[j], acc[i][j]);
        if (s2 == KS - 1) swrite(buf ^ 1, i);
      }
    }
  };
  // barrier without the vmcnt(0) drain of __syncthreads(): the loads of stage t + 2 stay in flight across it
  auto lds_barrier = []() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  if constexpr (DMA == 2) {
    if (T > 0) {
      issue(0, 0);
      wait_vm<0>();
      __syncthreads();
      for (int t = 0; t < T; ++t) {
        if (t + 1 < T) issue(t + 1, (t + 1) & 1);  // into the buffer every wave finished in stage t - 1
        const uint16_t* As = smem + (t & 1) * STAGE;
#pragma unroll
        for (int s2 = 0; s2 < KS; ++s2) {
          s16x8 bf[NT];
#pragma unroll
          for (int j = 0; j < NT; ++j) bf[j] = ld16(As + boff + (j * KS + s2) * 512);
          s16x8 af[2];
          af[0] = ld16(As + aoff0[s2]);
#pragma unroll
          for (int i = 0; i < MT; ++i) {
            if (i + 1 < MT) af[(i + 1) & 1] = ld16(As + aoff0[s2] + (i + 1) * 16 * BK);
#pragma unroll
            for (int j = 0; j < NT; ++j) acc[i][j] = mfma16(af[i & 1], bf[j], acc[i][j]);
          }
        }
        wait_vm<0>();
        lds_barrier();
      }
    }
  } else if (T > 0) {
    gload(0);
    if constexpr (DMA == 1) issue(0, 0);
#pragma unroll
    for (int i = 0; i < CH; ++i) swrite(0, i);
    gload(min(1, T - 1));
    if constexpr (DMA == 1) {
      if (T > 1) issue(1, 1);
    }
    __syncthreads();
    for (int t = 0; t < T; ++t) {
      compute(t & 1);
      gload(min(t + 2, T - 1));
      if constexpr (DMA == 1) {
        wait_vm<CH>();  // stage t+1's W DMA (issued a stage ago) landed; the X loads just issued stay out
        lds_barrier();
        if (t + 2 < T) issue(t + 2, t & 1);
      } else {
        lds_barrier();  // the other buffer is complete; every wave is done reading this one
      }
    }
  }

  // ---- epilogue (wave block rows wm * 128 .., columns wn * 128 ..)
  int ldy_e = ldy, ldr_e = ldr;
  asm volatile("" : "+s"(ldy_e), "+s"(ldr_e));
  const int rbase = m0 + wm * 128;
  const int cbase = n0 + wn * 128;
  if constexpr (SPLIT) {
    float* slab = ws + (size_t)split * M * N;
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = rbase + 16 * i + 4 * g + r;
        if (m < M) {
#pragma unroll
          for (int j = 0; j < NT; ++j) slab[(size_t)m * N + cbase + 16 * j + c] = acc[i][j][r];
        }
      }
  } else if constexpr (EPI == EPI_SILU) {
#pragma unroll
    for (int p = 0; p < NT / 2; ++p) {  // (gate tile 2p, up tile 2p+1) -> 16 output columns
      const int col = (cbase >> 1) + 16 * p + c;
      float bg = 0.f, bu = 0.f;
      if (bias != nullptr) {
        bg = bf2f(bias[cbase + 32 * p + c]);
        bu = bf2f(bias[cbase + 32 * p + 16 + c]);
      }
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = rbase + 16 * i + 4 * g + r;
          if (m < M) {
            const float v = silu(acc[i][2 * p][r] + bg) * (acc[i][2 * p + 1][r] + bu);
            if constexpr (OUT_F32)
              reinterpret_cast<float*>(Yv)[(size_t)m * ldy_e + col] = v;
            else
              reinterpret_cast<uint16_t*>(Yv)[(size_t)m * ldy_e + col] = f2bf(v);
          }
        }
    }
  } else {
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int col = cbase + 16 * j + c;
      const float bv = bias != nullptr ? bf2f(bias[col]) : 0.f;
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = rbase + 16 * i + 4 * g + r;
          if (m < M) {
            float v = acc[i][j][r] + bv;
            if constexpr (EPI == EPI_RESID) v += bf2f(R[(size_t)m * ldr_e + col]);
            if constexpr (OUT_F32)
              reinterpret_cast<float*>(Yv)[(size_t)m * ldy_e + col] = v;
            else
              reinterpret_cast<uint16_t*>(Yv)[(size_t)m * ldy_e + col] = f2bf(v);
          }
        }
    }
  }
}

template <int EPI, bool F32>
static void w4_launch(const uint16_t* X, int ldx, const uint16_t* W, const uint16_t* bias, const uint16_t* R, int ldr,
                      void* Y, int ldy, float* ws, int M, int N, int K, int S, bool reduce, hipStream_t st) {
  const int nwg = ((M + 255) / 256) * (N / 256) * S;
  if (S == 1) {
    auto kern = gemm_w4_kernel<EPI, F32, false>;
    static bool attr =
        hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, w4::SMEM) == hipSuccess;
    (void)attr;
    kern<<<nwg, 256, w4::SMEM, st>>>(X, ldx, W, bias, R, ldr, Y, ldy, nullptr, M, N, K, 1);
  } else {
    auto kern = gemm_w4_kernel<EPI, false, true>;
    static bool attr =
        hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, w4::SMEM) == hipSuccess;
    (void)attr;
    kern<<<nwg, 256, w4::SMEM, st>>>(X, ldx, W, bias, R, ldr, Y, ldy, ws, M, N, K, S);
    if (!reduce) return;  // slabs left for the consumer (fused reduce + residual + RMSNorm)
    const int ncol = EPI == EPI_SILU ? N / 2 : N;
    const long chunks = (long)M * (ncol / 8);
    int blocks = (int)((chunks + 255) / 256);
    if (blocks > 2048) blocks = 2048;
    splitk_reduce_kernel<EPI, F32><<<blocks, 256, 0, st>>>(ws, S, M, N, bias, R, ldr, Y, ldy);
  }
}

int launch_gemm_w4(const uint16_t* X, int ldx, const uint16_t* W, const uint16_t* bias, const uint16_t* R, int ldr,
                   void* Y, int ldy, bool out_f32, int epi, float* ws, long ws_elems, int M, int N, int K, int S,
                   bool reduce, hipStream_t s) {
  if (M <= 0) return 0;
  if (N % 256 != 0 || K % 128 != 0 || S < 1 || S > K / 64) return -1;
  if (S > 1 && (ws == nullptr || ws_elems < (long)S * M * N)) return -1;
  if (epi == EPI_SILU)
    out_f32 ? w4_launch<EPI_SILU, true>(X, ldx, W, bias, R, ldr, Y, ldy, ws, M, N, K, S, reduce, s)
            : w4_launch<EPI_SILU, false>(X, ldx, W, bias, R, ldr, Y, ldy, ws, M, N, K, S, reduce, s);
  else if (epi == EPI_RESID) {
    if (out_f32) return -1;
    w4_launch<EPI_RESID, false>(X, ldx, W, bias, R, ldr, Y, ldy, ws, M, N, K, S, reduce, s);
  } else
    out_f32 ? w4_launch<EPI_NONE, true>(X, ldx, W, bias, R, ldr, Y, ldy, ws, M, N, K, S, reduce, s)
            : w4_launch<EPI_NONE, false>(X, ldx, W, bias, R, ldr, Y, ldy, ws, M, N, K, S, reduce, s);
  return 0;
}

}  // namespace xot

// Causal self-attention for the training step (flash-style, no S x S matrix), MFMA 16x16x32 bf16.
//
// Tensors are token-major slices of the projection outputs: Q [B*L, ldq] holding H heads of DH,
// K / V [B*L, ldk / ldv] holding Hkv heads (GQA: query head h reads KV head h / (H / Hkv)).
// Sequences are right-padded to L; causality alone keeps valid queries off padded keys.
//
// Operands that MFMA reads "by column": V for P.V comes from a pre-transposed [B, heads, DH, Lp] image
// (attn_train_transpose_kernel); the backward's K (dS.K) and Q / dO (dK / dV products) are read transposed out of
// the row tiles already in LDS (ds_read_b64_tr_b16, the v2 kernels; v1 staged transposed images of them too).
// The next tile is loaded into registers under the current tile's math.
//
//  fwd   grid (L/64, H, B): 4 waves x 16 query rows.  Per 64-key tile: K rows and V^T staged in LDS,
//        S = Q.K^T, online softmax in the log2 domain, P through LDS into P.V.  Writes O and the
//        per-row log2-sum-exp (lse2 = max + log2 sum, scores pre-scaled by scale*log2(e)).
//  dq    grid (H, L/64, B): recomputes P from lse2, dP = dO.V^T, dS = P (dP - delta); dQ += dS.K.
//        Also computes delta = rowsum(dO * O) for its rows and stores it for the dK/dV pass.  v2: S^T / dP^T
//        with the key on the accumulator row, dS^T stays in registers as the B operand of dQ^T += K^T.dS^T.
//  dkdv  grid (H, L/128, B): 8 waves x 16 keys per query head; sweeps the query tiles >= its key tile; fp32
//        partials per query head, summed over the GQA group by attn_train_dkdv_reduce_kernel.  v1: S^T, dP^T
//        with the query on the lane, P^T / dS^T through LDS into dV += P^T.dO, dK += dS^T.Q; v2: S, dP with
//        the query on the accumulator row, P / dS stay in registers as the B operands of dV^T / dK^T.
//
// Replaces torch SDPA in the reference-parity train step (the reference never implemented training:
// xotorch/inference/inference_engine.py:34-35; the torchtune attention it would have used is
// MultiHeadAttention via xotorch/inference/torch/models/general_mha.py:77-120).
#include "common.h"
#include "kernels.h"

namespace xot {

namespace {
constexpr int TT = 64;  // query / key tile
constexpr float NEG = -1e30f;
constexpr float L2E = 1.4426950408889634f;

__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// Register-staged tile copies (256 threads, 16-byte chunks): load() issues the global loads into registers
// (in flight under the current tile's math), store() writes them to LDS after the barrier.
//   rows tile:  [64 tokens][DH] of a token-major source (ld elements per token), tokens clamped to L-1
//   trans tile: [DH][64 tokens] of a pre-transposed [.., DH, Lp] image (zero past L)
template <int DH, int NT = 256>
struct RowsTile {
  static constexpr int N = TT * DH / 8 / NT;  // chunks per thread
  static_assert(N >= 1 && TT * DH / 8 % NT == 0, "tile / thread count");
  s16x8 v[N];
  __device__ __forceinline__ void load(const uint16_t* __restrict__ src, long ld, int row0, int L) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int q = threadIdx.x + NT * i, r = q / (DH / 8), cc = q % (DH / 8);
      v[i] = ld16(src + (long)min(row0 + r, L - 1) * ld + cc * 8);
    }
  }
  template <int RLD>
  __device__ __forceinline__ void store(uint16_t* dst) const {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int q = threadIdx.x + NT * i, r = q / (DH / 8), cc = q % (DH / 8);
      st16(dst + r * RLD + cc * 8, v[i]);
    }
  }
};
template <int DH, int NT = 256>
struct TransTile {
  static constexpr int N = DH * TT / 8 / NT;
  static_assert(N >= 1 && DH * TT / 8 % NT == 0, "tile / thread count");
  s16x8 v[N];
  __device__ __forceinline__ void load(const uint16_t* __restrict__ srcT, int Lp, int tok0) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int q = threadIdx.x + NT * i, d = q / (TT / 8), cc = q % (TT / 8);
      v[i] = ld16(srcT + (long)d * Lp + tok0 + cc * 8);
    }
  }
  template <int TLD>
  __device__ __forceinline__ void store(uint16_t* dst) const {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int q = threadIdx.x + NT * i, d = q / (TT / 8), cc = q % (TT / 8);
      st16(dst + d * TLD + cc * 8, v[i]);
    }
  }
};
}  // namespace

// ---------------------------------------------------------------------------------------- forward
// Each wave owns FRB blocks of 16 query rows (4 waves x FRB x 16 = the workgroup's query tile): every K /
// V^T fragment read from LDS feeds FRB MFMAs.  FRB = 2 halves the LDS reads per MFMA but also halves the
// grid (512 workgroups for 32 heads at L = 2048, under two per CU), which measured slower (116 vs 103 us).
constexpr int FRB = 1, FQT = 64 * FRB;  // FRB = 2 measured slower at L = 2048 (half the workgroups)
// CAUSAL = false: every query attends to all L keys (the bidirectional attention of the CLIP vision tower).
template <int DH, bool CAUSAL = true>
__global__ __launch_bounds__(256) void attn_train_fwd_kernel(const uint16_t* __restrict__ Q, long ldq,
                                                             const uint16_t* __restrict__ K, long ldk,
                                                             const uint16_t* __restrict__ VT, int Lp,
                                                             uint16_t* __restrict__ O, long ldo,
                                                             float* __restrict__ lse2, int L, int H, int Hkv,
                                                             float scale) {
  constexpr int KS = DH / 32, NDT = DH / 16;
  constexpr int KLD = DH + 8, VLD = TT + 8, PLD = TT + 8;
  __shared__ __attribute__((aligned(16))) uint16_t ks[TT * KLD];
  __shared__ __attribute__((aligned(16))) uint16_t vt[DH * VLD];
  __shared__ __attribute__((aligned(16))) uint16_t pl[4][FRB][16 * PLD];
  // query tiles are the slowest grid dimension, heaviest (most key tiles under the causal mask) first
  const int h = blockIdx.x, qt = gridDim.y - 1 - blockIdx.y, b = blockIdx.z;
  const int kvh = h / (H / Hkv);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, c = lane & 15;
  const int q0 = qt * FQT, qrow = q0 + 16 * FRB * wave;  // row block rb: rows qrow + 16 rb ..
  const int ktl = CAUSAL ? min((L + TT - 1) / TT, (q0 + FQT + TT - 1) / TT) - 1  // last key tile under the mask
                         : (L + TT - 1) / TT - 1;
  const uint16_t* Kb = K + (long)b * L * ldk + kvh * DH;
  const uint16_t* VTb = VT + ((long)b * Hkv + kvh) * DH * Lp;
  const float sl = scale * L2E;

  s16x8 qf[FRB][KS];
#pragma unroll
  for (int rb = 0; rb < FRB; ++rb) {
    const uint16_t* qp = Q + ((long)b * L + min(qrow + 16 * rb + c, L - 1)) * ldq + h * DH + 8 * g;
#pragma unroll
    for (int s2 = 0; s2 < KS; ++s2) qf[rb][s2] = ld16(qp + 32 * s2);
  }
  float m[FRB][4], l[FRB][4];
  f32x4 o[FRB][NDT];
#pragma unroll
  for (int rb = 0; rb < FRB; ++rb) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      m[rb][r] = NEG;
      l[rb][r] = 0.f;
    }
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) o[rb][dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  RowsTile<DH> kr;
  TransTile<DH> vr;
  kr.load(Kb, ldk, 0, L);
  vr.load(VTb, Lp, 0);
  for (int kt = 0; kt <= ktl; ++kt) {
    const int k0 = kt * TT;
    __syncthreads();  // every wave is done with the previous tile
    kr.template store<KLD>(ks);
    vr.template store<VLD>(vt);
    __syncthreads();
    if (kt < ktl) {  // next tile in flight under this tile's math
      kr.load(Kb, ldk, k0 + TT, L);
      vr.load(VTb, Lp, k0 + TT);
    }
    f32x4 sc[FRB][4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
#pragma unroll
      for (int rb = 0; rb < FRB; ++rb) sc[rb][t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s2 = 0; s2 < KS; ++s2) {
        const s16x8 kb = ld16(ks + (16 * t + c) * KLD + 32 * s2 + 8 * g);
#pragma unroll
        for (int rb = 0; rb < FRB; ++rb) sc[rb][t] = mfma16(qf[rb][s2], kb, sc[rb][t]);
      }
    }
#pragma unroll
    for (int rb = 0; rb < FRB; ++rb) {
      float mt[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) mt[r] = NEG;
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = k0 + 16 * t + c, qi = qrow + 16 * rb + 4 * g + r;
          const float v = ((!CAUSAL || key <= qi) && key < L) ? sc[rb][t][r] * sl : -INFINITY;
          sc[rb][t][r] = v;
          mt[r] = fmaxf(mt[r], v);
        }
      float alpha[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        mt[r] = group16_max(mt[r]);
        const float mn = fmaxf(m[rb][r], mt[r]);
        alpha[r] = exp2f(m[rb][r] - mn);
        m[rb][r] = mn;
        l[rb][r] *= alpha[r];
      }
      uint16_t* pw = pl[wave][rb];
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float p = exp2f(sc[rb][t][r] - m[rb][r]);
          l[rb][r] += p;
          pw[(4 * g + r) * PLD + 16 * t + c] = f2bf(p);
        }
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
        for (int r = 0; r < 4; ++r) o[rb][dt][r] *= alpha[r];
    }
    wave_sync_lds();
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      s16x8 pa[FRB];
#pragma unroll
      for (int rb = 0; rb < FRB; ++rb) pa[rb] = ld16(pl[wave][rb] + c * PLD + 32 * kk + 8 * g);
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
        const s16x8 vb = ld16(vt + (16 * dt + c) * VLD + 32 * kk + 8 * g);
#pragma unroll
        for (int rb = 0; rb < FRB; ++rb) o[rb][dt] = mfma16(pa[rb], vb, o[rb][dt]);
      }
    }
  }
#pragma unroll
  for (int rb = 0; rb < FRB; ++rb)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float ls = group16_sum(l[rb][r]);
      const int qi = qrow + 16 * rb + 4 * g + r;
      if (qi >= L) continue;
      const float inv = ls > 0.f ? 1.f / ls : 0.f;
      uint16_t* op = O + ((long)b * L + qi) * ldo + h * DH + c;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) op[16 * dt] = f2bf(o[rb][dt][r] * inv);
      if (c == 0) lse2[((long)b * H + h) * L + qi] = m[rb][r] + log2f(ls);
    }
}

// ---------------------------------------------------------------------------------------- forward, v2
// The causal forward on the schedule of the serving prefill kernel (csrc/attention.hip attn_prefill_v2_kernel,
// 745-932 TF/s vs ~375 for attn_train_fwd_kernel above): one workgroup = 8 waves = 256 rows (token, head-in-
// group) of one (sequence, KV head), two 16-row blocks per wave so every K / V^T fragment read from LDS feeds
// two MFMAs; S^T = K . Q^T with the K rows permuted so the probabilities land in the B-operand layout of
// O^T += V^T . P^T (softmax lane-local but for two shuffles of the page max, no LDS round trip for P); K rows
// (token-major, stride ldk) and V^T rows (the [B, Hkv, DH, Lp] image) arrive by LDS-DMA in a three-page ring,
// XOR-swizzled through the source addresses so every fragment read is bank-conflict free.  Writes O and the
// same per-row lse2 (log2 domain) as attn_train_fwd_kernel, so the dQ / dK dV passes are unchanged.
template <int DH>
__device__ __forceinline__ int tf2_kswz(int r) {  // K-row granule swizzle (the prefill kernel's searched map)
  return DH == 128 ? (3 * (r & 1)) | (((r >> 1) & 1) << 2) | (((r >> 3) & 1) << 3)
                   : (r & 1) | (((r >> 1) & 1) << 1) | (((r >> 3) & 1) << 2);
}

template <int DH>
__global__ __launch_bounds__(512, 1) void attn_train_fwd_v2_kernel(const uint16_t* __restrict__ Q, long ldq,
                                                                   const uint16_t* __restrict__ K, long ldk,
                                                                   const uint16_t* __restrict__ VT, int Lp,
                                                                   uint16_t* __restrict__ O, long ldo,
                                                                   float* __restrict__ lse2, int L, int H, int Hkv,
                                                                   float sl) {
  constexpr int KS = DH / 32, NDT = DH / 16, KGPR = DH / 8;
  constexpr int PAGE_EL = TT * DH;          // elements of one K (or V^T) page
  constexpr int NCH = 2 * PAGE_EL / 512;    // 1 KB LDS-DMA chunks per page (K then V^T)
  static_assert(NCH % 8 == 0, "chunks split over 8 waves");
  constexpr int CPW = NCH / 8;
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];  // [3][K page | V^T page]

  int tile, kvh, b;
  {  // bijective XCD remap: the tiles of one (sequence, KV head) on one XCD; heaviest (latest rows) first
    const int nwg = gridDim.x * gridDim.y * gridDim.z;
    int lin = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    const int xcd = lin & 7, qq = nwg >> 3, rr = nwg & 7;
    lin = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (lin >> 3);
    tile = gridDim.x - 1 - lin % gridDim.x;
    lin /= gridDim.x;
    kvh = lin % gridDim.y;
    b = lin / gridDim.y;
  }
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c = lane & 15;
  const int G = H / Hkv, nrows = L * G, row0 = tile * 256;
  if (row0 >= nrows) return;  // whole workgroup exits together

  // Q^T fragments (B operand: k = dims, n = rows): lane (g, c) holds row c of block blk, dims 32 s + 8 g .. +8
  s16x8 qf[2][KS];
  int qpos[2];
#pragma unroll
  for (int blk = 0; blk < 2; ++blk) {
    const int row = row0 + 32 * wave + 16 * blk + c;
    const bool ok = row < nrows;
    const int ti = ok ? row / G : 0, hi = ok ? row % G : 0;
    qpos[blk] = ok ? ti : -1;
    const uint16_t* qp = Q + ((long)b * L + ti) * ldq + (kvh * G + hi) * DH + 8 * g;
#pragma unroll
    for (int s2 = 0; s2 < KS; ++s2) {
      const s16x8 v = ld16(qp + 32 * s2);
      qf[blk][s2] = ok ? v : s16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
  }
  const int last_row = min(nrows, row0 + 256) - 1;
  const int npages = (last_row / G) / TT + 1;
  const int wlast = min(nrows - 1, row0 + 32 * wave + 31);
  const int wmax = wlast >= row0 + 32 * wave ? wlast / G : -1;  // this wave's last key (causal)
  const int wmin = (row0 + 32 * wave) / G;                       // ... and its first row's

  float m[2] = {NEG, NEG}, l[2] = {0.f, 0.f};
  f32x4 o[2][NDT];
#pragma unroll
  for (int blk = 0; blk < 2; ++blk)
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) o[blk][dt] = f32x4{0.f, 0.f, 0.f, 0.f};

  const uint16_t* Kb = K + (long)b * L * ldk + kvh * DH;
  const uint16_t* VTb = VT + ((long)b * Hkv + kvh) * DH * Lp;
  auto issue = [&](int p, int buf) {
    uint16_t* dst = smem + buf * 2 * PAGE_EL;
#pragma unroll
    for (int i = 0; i < CPW; ++i) {
      const int ch = wave * CPW + i;
      const int P = (ch % (NCH / 2)) * 64 + lane;  // granule of the K or V^T page image
      const uint16_t* src;
      if (ch < NCH / 2) {
        const int r = P / KGPR, j = (P % KGPR) ^ tf2_kswz<DH>(r);
        src = Kb + (long)min(p * TT + r, L - 1) * ldk + j * 8;  // keys past L: masked (key > every row)
      } else {
        const int r = P >> 3, j = (P & 7) ^ (r & 7);  // V^T rows: 64 keys = 8 granules (zero past L)
        src = VTb + (long)r * Lp + p * TT + j * 8;
      }
      __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)(dst + ch * 512), 16, 0, 0);
    }
  };
  int kofs[4][KS];  // fragment addresses (elements inside a page image), fixed per lane
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int r = 32 * (j >> 1) + 8 * (c >> 2) + 4 * (j & 1) + (c & 3);
#pragma unroll
    for (int s2 = 0; s2 < KS; ++s2) kofs[j][s2] = r * DH + 8 * ((4 * s2 + g) ^ tf2_kswz<DH>(r));
  }
  int vofs[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) vofs[kk] = c * TT + 8 * ((4 * kk + g) ^ (c & 7));

  // S^T, causal mask and the online softmax of one page -> P^T fragments and the rescale factors
  auto score = [&](const uint16_t* Ks, int key0, s16x8 (&pf)[2][2], float (&alpha)[2]) {
    f32x4 st[2][4];
#pragma unroll
    for (int blk = 0; blk < 2; ++blk)
#pragma unroll
      for (int j = 0; j < 4; ++j) st[blk][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    constexpr int KPF = 4, NKS = 4 * KS;  // K fragments KPF steps ahead of their MFMAs
    s16x8 ka[KPF];
#pragma unroll
    for (int t = 0; t < KPF - 1; ++t) ka[t] = ld16(Ks + kofs[t & 3][t >> 2]);
#pragma unroll
    for (int t = 0; t < NKS; ++t) {
      if (t + KPF - 1 < NKS) ka[(t + KPF - 1) % KPF] = ld16(Ks + kofs[(t + KPF - 1) & 3][(t + KPF - 1) >> 2]);
      const int j = t & 3, s2 = t >> 2;
      st[0][j] = mfma16(ka[t % KPF], qf[0][s2], st[0][j]);
      st[1][j] = mfma16(ka[t % KPF], qf[1][s2], st[1][j]);
      __builtin_amdgcn_sched_barrier(0);
    }
    const bool need_mask = key0 + TT - 1 > wmin;  // wave-uniform
#pragma unroll
    for (int blk = 0; blk < 2; ++blk) {
      if (need_mask) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int key = key0 + 32 * (j >> 1) + 8 * g + 4 * (j & 1) + r;
            st[blk][j][r] = key <= qpos[blk] ? st[blk][j][r] : -INFINITY;
          }
      }
      float mt = NEG;
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) mt = fmaxf(mt, st[blk][j][r]);
      mt = fmaxf(mt, __shfl_xor(mt, 16, 64));
      mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
      const float mn = fmaxf(m[blk], mt * sl);
      alpha[blk] = __builtin_amdgcn_exp2f(m[blk] - mn);
      m[blk] = mn;
      float ls = 0.f;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        u32x4 pw;
#pragma unroll
        for (int e = 0; e < 8; e += 2) {
          const float p0 = __builtin_amdgcn_exp2f(fmaf(st[blk][2 * kk + (e >> 2)][e & 3], sl, -mn));
          const float p1 = __builtin_amdgcn_exp2f(fmaf(st[blk][2 * kk + (e >> 2)][(e & 3) + 1], sl, -mn));
          pw[e >> 1] = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t{p0, p1}), bf16x2_t));
          ls += p0 + p1;
        }
        pf[blk][kk] = __builtin_bit_cast(s16x8, pw);
      }
      l[blk] = l[blk] * alpha[blk] + ls;
    }
  };
  // O^T = alpha O^T + V^T . P^T for one page
  auto accumulate = [&](const uint16_t* Vs, const s16x8 (&pf)[2][2], const float (&alpha)[2]) {
    if (__ballot(alpha[0] != 1.f || alpha[1] != 1.f)) {  // no row's max moved: no rescale (wave-uniform)
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          o[0][dt][r] *= alpha[0];
          o[1][dt][r] *= alpha[1];
        }
    }
    constexpr int VPF = 3;  // V^T fragments VPF dim tiles ahead of their MFMAs
    s16x8 va[VPF][2];
#pragma unroll
    for (int t = 0; t < VPF - 1; ++t)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) va[t][kk] = ld16(Vs + vofs[kk] + 16 * t * TT);
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
      if (dt + VPF - 1 < NDT) {
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) va[(dt + VPF - 1) % VPF][kk] = ld16(Vs + vofs[kk] + 16 * (dt + VPF - 1) * TT);
      }
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        o[0][dt] = mfma16(va[dt % VPF][kk], pf[0][kk], o[0][dt]);
        o[1][dt] = mfma16(va[dt % VPF][kk], pf[1][kk], o[1][dt]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // three-page ring, two pages in flight: page p + 2 is issued once every wave is past page p - 1
  issue(0, 0);
  if (npages > 1) issue(1, 1);
  for (int p = 0; p < npages; ++p) {
    const int buf = p % 3;
    if (p + 1 < npages)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(CPW) : "memory");  // this wave's share of page p landed
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (p + 2 < npages) issue(p + 2, (p + 2) % 3);
    const int key0 = p * TT;
    if (key0 > wmax) continue;  // wave-uniform: every row of this wave is before the page (causal)
    const uint16_t* Ks = smem + buf * 2 * PAGE_EL;
    s16x8 pf[2][2];
    float alpha[2];
    score(Ks, key0, pf, alpha);
    accumulate(Ks + PAGE_EL, pf, alpha);
  }

  // o[blk][dt][r] = O[row c of block blk][dim 16 dt + 4 g + r]
#pragma unroll
  for (int blk = 0; blk < 2; ++blk) {
    float ls = l[blk];
    ls += __shfl_xor(ls, 16, 64);
    ls += __shfl_xor(ls, 32, 64);
    const int row = row0 + 32 * wave + 16 * blk + c;
    if (row < nrows) {
      const int ti = row / G, h = kvh * G + row % G;
      uint16_t* op = O + ((long)b * L + ti) * ldo + h * DH + 4 * g;
      const float inv = ls > 0.f ? 1.f / ls : 0.f;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
        s16x4 v;
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = (short)f2bf(o[blk][dt][r] * inv);
        *reinterpret_cast<s16x4*>(op + 16 * dt) = v;
      }
      if (g == 0) lse2[((long)b * H + h) * L + ti] = m[blk] + log2f(ls);
    }
  }
}

// ---------------------------------------------------------------------------------------- dK, dV
// DKW = 8 waves: 128 keys per workgroup share each staged query tile (2 waves per SIMD, so one wave's
// LDS reads and exp2 hide under the other's MFMAs; with 4 waves the LDS footprint left one wave per SIMD)
constexpr int DKW = 8, DKT = 16 * DKW;
// dK = scale * sum_h wk[h], dV = sum_h wv[h]  ([G][rows][cols] fp32 -> bf16 row views)
__global__ __launch_bounds__(256) void attn_train_dkdv_reduce_kernel(const float* __restrict__ wk,
                                                                     const float* __restrict__ wv, int G, long rows,
                                                                     int cols, float scale, uint16_t* __restrict__ dK,
                                                                     long lddk, uint16_t* __restrict__ dV, long lddv) {
  const long n4 = rows * cols / 4, slab = rows * cols;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    f32x4 a = f32x4{0.f, 0.f, 0.f, 0.f}, v = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int h = 0; h < G; ++h) {
      a += *reinterpret_cast<const f32x4*>(wk + h * slab + 4 * i);
      v += *reinterpret_cast<const f32x4*>(wv + h * slab + 4 * i);
    }
    const long row = 4 * i / cols, col = 4 * i % cols;
    s16x4 ka, va;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      ka[e] = (short)f2bf(a[e] * scale);
      va[e] = (short)f2bf(v[e]);
    }
    *reinterpret_cast<s16x4*>(dK + row * lddk + col) = ka;
    *reinterpret_cast<s16x4*>(dV + row * lddv + col) = va;
  }
}

// ---------------------------------------------------------------------------------------- transpose
// X [B*L, ldx] token-major, n heads of DH -> XT [B, n, DH, Lp] (tokens contiguous, zero for t >= L).
template <int DH>
__global__ __launch_bounds__(256) void attn_train_transpose_kernel(const uint16_t* __restrict__ X, long ldx,
                                                                   uint16_t* __restrict__ XT, int L, int Lp, int n) {
  constexpr int TLD = TT + 8;
  __shared__ __attribute__((aligned(16))) uint16_t tl[DH * TLD];
  const int t0 = blockIdx.x * TT, hd = blockIdx.y, b = blockIdx.z;
  for (int q = threadIdx.x; q < TT * (DH / 8); q += 256) {  // read 64 tokens x DH (16-B loads)
    const int r = q / (DH / 8), cc = q % (DH / 8);
    s16x8 v = s16x8{0, 0, 0, 0, 0, 0, 0, 0};
    if (t0 + r < L) v = ld16(X + ((long)b * L + t0 + r) * ldx + hd * DH + cc * 8);
#pragma unroll
    for (int e = 0; e < 8; ++e) tl[(cc * 8 + e) * TLD + r] = (uint16_t)v[e];
  }
  __syncthreads();
  uint16_t* out = XT + (((long)b * n + hd) * DH) * Lp + t0;
  for (int q = threadIdx.x; q < DH * (TT / 8); q += 256) {  // write DH rows x 64 tokens (16-B stores)
    const int d = q / (TT / 8), cc = q % (TT / 8);
    st16(out + (long)d * Lp + cc * 8, ld16(tl + d * TLD + cc * 8));
  }
}

// dK / dV without the P^T / dS^T round trip through LDS (v2).  S = Q.K^T and dP = dO.V^T are computed with the
// query on the accumulator row (lane (g, c) holds queries 16 t + 4 g + r of key c), so two 16-query sub-tiles
// give a lane the 8 values of B-operand rows 8 g .. 8 g + 7 of dV^T += dO^T . P and dK^T += Q^T . dS -- in
// the k order "sub-tile 2 kk rows 4 g .. 4 g + 3, then sub-tile 2 kk + 1 rows 4 g .. 4 g + 3".  That is the
// order two transposed LDS reads (tr_frag) deliver the Q^T / dO^T A fragments in, straight from the row-major
// Q / dO tiles the S and dP products read: no transposed images in HBM or LDS.  v1 stored 32 two-byte P^T / dS^T
// values per lane and query tile and read them back, and staged Q^T / dO^T tiles besides; v2 needs a third of
// v1's LDS.
typedef __attribute__((address_space(3))) s16x4* lds_s16x4_t;
// The A operand X^T[col 16 dt + c][rows in the permuted order] of a row-major LDS tile X [64][ld]: two
// ds_read_b64_tr_b16 (4 rows x 16 columns each, column c to lane c of the 16-lane group g): rows 32 kk + 4 g .. +3
// (elements 0..3) and rows 32 kk + 16 + 4 g .. +3 (elements 4..7).  Lane 4 q + p of the group addresses row q,
// columns 4 p .. 4 p + 3 of its block.  A row stride of 8 (mod 64) dwords keeps both reads conflict-free.
__device__ __forceinline__ s16x8 tr_frag(const uint16_t* X, int ld, int kk, int dt, int g, int c) {
  const uint16_t* p = X + (32 * kk + 4 * g + (c >> 2)) * ld + 16 * dt + 4 * (c & 3);
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t)(p));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t)(p + 16 * ld));
  return s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}
// Row stride of those tiles: DH + 16 elements = 72 dwords (DH 128) or 40 (DH 64, 192) mod 64, so the 8 rows a
// 32-lane half reads sit on 8 distinct 8-bank groups (and the 16x16x32 row reads stay conflict-free too).
__host__ __device__ constexpr int tr_ld(int dh) { return dh + 16; }

template <int DH>
__global__ __launch_bounds__(64 * DKW) void attn_train_dkdv_v2_kernel(const uint16_t* __restrict__ Q, long ldq,
                                                                   const uint16_t* __restrict__ QT,
                                                                   const uint16_t* __restrict__ K, long ldk,
                                                                   const uint16_t* __restrict__ V, long ldv,
                                                                   const uint16_t* __restrict__ dO, long lddo,
                                                                   const uint16_t* __restrict__ dOT, int Lp,
                                                                   const float* __restrict__ lse2,
                                                                   const float* __restrict__ delta,
                                                                   float* __restrict__ wk, float* __restrict__ wv,
                                                                   int L, int H, int Hkv, float scale, int hpw) {
  constexpr int KS = DH / 32, NDT = DH / 16;
  constexpr int RLD = tr_ld(DH);
  extern __shared__ __attribute__((aligned(16))) uint16_t sm[];
  uint16_t* qs = sm;                 // Q rows       [64][RLD] (row reads for S, transposed reads for dK)
  uint16_t* ds_ = qs + TT * RLD;     // dO rows      [64][RLD] (row reads for dP, transposed reads for dV)
  float* ld_ = reinterpret_cast<float*>(ds_ + TT * RLD);  // lse2[64], delta[64]
  // hpw query heads of one GQA group per workgroup (their dK / dV sum in the accumulators): G / hpw partial
  // slabs for the reduce kernel instead of G.  2 at G = 4 keeps 512 workgroups of 64 .. 4 query tiles, which
  // heaviest-first scheduling still balances over 256 CUs; 4 would leave one workgroup per CU, 128 vs 8 tiles.
  const int G = H / Hkv;
  const int hq = blockIdx.x * hpw, kvh = hq / G, hh = (hq % G) / hpw, kt = blockIdx.y, b = blockIdx.z;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, c = lane & 15;
  const int k0 = kt * DKT, krow = k0 + 16 * wave;
  const float sl = scale * L2E;
  const int qt0 = k0 / TT;
  const int nq = (L + TT - 1) / TT, iters = (nq - qt0) * hpw;  // (head, query tile) pairs, head-major
  const int per = nq - qt0;
  const int key = krow + c;  // this lane's key (B-operand column of every product)

  RowsTile<DH, 64 * DKW> qr, dr;
  float lsv = 0.f, dlv = 0.f;
  auto load = [&](int it) {
    const int h = hq + it / per, q0 = (qt0 + it % per) * TT;
    qr.load(Q + (long)b * L * ldq + h * DH, ldq, q0, L);
    dr.load(dO + (long)b * L * lddo + h * DH, lddo, q0, L);
    if (threadIdx.x < TT) {
      const long idx = ((long)b * H + h) * L + min(q0 + (int)threadIdx.x, L - 1);
      lsv = lse2[idx];
      dlv = delta[idx];
    }
  };

  s16x8 kf[KS], vf[KS];  // B operands: lane (g, c) = key c, dims 32 s + 8 g .. +7
  {
    const long row = (long)b * L + min(key, L - 1);
    const uint16_t* kp = K + row * ldk + kvh * DH + 8 * g;
    const uint16_t* vp = V + row * ldv + kvh * DH + 8 * g;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      kf[s] = ld16(kp + 32 * s);
      vf[s] = ld16(vp + 32 * s);
    }
  }
  f32x4 dkT[NDT], dvT[NDT];  // [dim 16 dt + 4 g + r][key c]
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) dkT[dt] = dvT[dt] = f32x4{0.f, 0.f, 0.f, 0.f};

  // The row constants ride in as the accumulators' initial values (LDS: -lse2 / sl, -delta per query row), so
  // S' = Q.K^T - lse2 / sl and dP' = dO.V^T - delta leave their MFMA chains ready: p = exp2(sl S') and
  // dS = p dP' cost one multiply each.  Only tiles that straddle the diagonal or the sequence end are masked.
  const float isl = 1.f / sl;
  auto tile = [&](const int q0, auto masked) {
    constexpr bool MASK = decltype(masked)::value;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {  // 32 queries: sub-tiles 2 kk and 2 kk + 1
      uint32_t pw[4], sw[4];
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) {
        const int t = 2 * kk + tt;
        f32x4 st = *reinterpret_cast<const f32x4*>(ld_ + 16 * t + 4 * g);
        f32x4 dpt = *reinterpret_cast<const f32x4*>(ld_ + TT + 16 * t + 4 * g);
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          st = mfma16(ld16(qs + (16 * t + c) * RLD + 32 * s + 8 * g), kf[s], st);
          dpt = mfma16(ld16(ds_ + (16 * t + c) * RLD + 32 * s + 8 * g), vf[s], dpt);
        }
        float p[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          p[r] = __builtin_amdgcn_exp2f(st[r] * sl);
          if constexpr (MASK) {
            const int qi = q0 + 16 * t + 4 * g + r;
            if (!(key <= qi && qi < L)) p[r] = 0.f;
          }
        }
        pw[2 * tt] = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t{p[0], p[1]}), bf16x2_t));
        pw[2 * tt + 1] = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t{p[2], p[3]}), bf16x2_t));
        sw[2 * tt] = __builtin_bit_cast(uint32_t,
                                        __builtin_convertvector((f32x2_t{p[0] * dpt[0], p[1] * dpt[1]}), bf16x2_t));
        sw[2 * tt + 1] = __builtin_bit_cast(uint32_t,
                                            __builtin_convertvector((f32x2_t{p[2] * dpt[2], p[3] * dpt[3]}), bf16x2_t));
      }
      const s16x8 pa = __builtin_bit_cast(s16x8, u32x4{pw[0], pw[1], pw[2], pw[3]});
      const s16x8 sa = __builtin_bit_cast(s16x8, u32x4{sw[0], sw[1], sw[2], sw[3]});
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
        dvT[dt] = mfma16(tr_frag(ds_, RLD, kk, dt, g, c), pa, dvT[dt]);
        dkT[dt] = mfma16(tr_frag(qs, RLD, kk, dt, g, c), sa, dkT[dt]);
      }
    }
  };

  if (iters > 0) load(0);
  for (int it = 0; it < iters; ++it) {
    const int q0 = (qt0 + it % per) * TT;
    __syncthreads();
    qr.template store<RLD>(qs);
    dr.template store<RLD>(ds_);
    if (threadIdx.x < TT) {
      ld_[threadIdx.x] = -lsv * isl;
      ld_[TT + threadIdx.x] = -dlv;
    }
    __syncthreads();
    if (it + 1 < iters) load(it + 1);
    if (q0 >= krow + 15 && q0 + TT <= L)  // wave-uniform: every query of the tile sees all 16 keys of this wave
      tile(q0, std::false_type{});
    else
      tile(q0, std::true_type{});
  }
  if (key >= L) return;
  const long slab = (long)hh * ((long)gridDim.z * L) * (Hkv * DH);
  const long off = slab + ((long)b * L + key) * (Hkv * DH) + kvh * DH + 4 * g;
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) {
    *reinterpret_cast<f32x4*>(wk + off + 16 * dt) = dkT[dt];
    *reinterpret_cast<f32x4*>(wv + off + 16 * dt) = dvT[dt];
  }
}

// dQ without the dS round trip through LDS (v2, the dkdv v2 idea on the query side): S^T = K.Q^T and
// dP^T = V.dO^T put the key on the accumulator row (lane (g, c) holds keys 16 t + 4 g + r of query c), two
// 16-key sub-tiles give a lane the 8 B-operand values of dQ^T += K^T . dS^T, and K^T is staged in the matching
// permuted key order.  Each lane owns one query, so lse2 / delta are lane scalars.
template <int DH>
__global__ __launch_bounds__(256) void attn_train_dq_v2_kernel(const uint16_t* __restrict__ Q, long ldq,
                                                               const uint16_t* __restrict__ K, long ldk,
                                                               const uint16_t* __restrict__ KT,
                                                               const uint16_t* __restrict__ V, long ldv,
                                                               const uint16_t* __restrict__ O, long ldo,
                                                               const uint16_t* __restrict__ dO, long lddo, int Lp,
                                                               const float* __restrict__ lse2,
                                                               float* __restrict__ delta, uint16_t* __restrict__ dQ,
                                                               long lddq, int L, int H, int Hkv, float scale) {
  constexpr int KS = DH / 32, NDT = DH / 16;
  constexpr int KLD = tr_ld(DH);
  __shared__ __attribute__((aligned(16))) uint16_t ks[TT * KLD];   // K rows (row reads for S^T, transposed for dQ)
  __shared__ __attribute__((aligned(16))) uint16_t vs[TT * KLD];   // V rows
  const int h = blockIdx.x, qt = gridDim.y - 1 - blockIdx.y, b = blockIdx.z;
  const int kvh = h / (H / Hkv);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, c = lane & 15;
  const int q0 = qt * TT, qrow = q0 + 16 * wave, qi = qrow + c;  // this lane's query
  const uint16_t* Kb = K + (long)b * L * ldk + kvh * DH;
  const uint16_t* Vb = V + (long)b * L * ldv + kvh * DH;
  const float sl = scale * L2E;

  RowsTile<DH> kr, vr;
  kr.load(Kb, ldk, 0, L);
  vr.load(Vb, ldv, 0, L);

  s16x8 qf[KS], df[KS];  // B operands: lane (g, c) = query c, dims 32 s + 8 g .. +7
  float dsum = 0.f;
  {
    const long row = (long)b * L + min(qi, L - 1);
    const uint16_t* qp = Q + row * ldq + h * DH + 8 * g;
    const uint16_t* dp = dO + row * lddo + h * DH + 8 * g;
    const uint16_t* opp = O + row * ldo + h * DH + 8 * g;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      qf[s] = ld16(qp + 32 * s);
      df[s] = ld16(dp + 32 * s);
      const s16x8 ov = ld16(opp + 32 * s);
#pragma unroll
      for (int e = 0; e < 8; ++e) dsum += bf2f(df[s][e]) * bf2f(ov[e]);
    }
  }
  dsum += __shfl_xor(dsum, 16, 64);  // delta of query c, in every lane group
  dsum += __shfl_xor(dsum, 32, 64);
  if (g == 0 && qi < L) delta[((long)b * H + h) * L + qi] = dsum;
  const float lse = lse2[((long)b * H + h) * L + min(qi, L - 1)];
  f32x4 dqT[NDT];  // [dim 16 dt + 4 g + r][query c]
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) dqT[dt] = f32x4{0.f, 0.f, 0.f, 0.f};

  // row constants as the accumulators' initial values (the dK / dV kernel's scheme; here they are lane scalars):
  // p = exp2(sl (S - lse2 / sl)), dS = p (dP - delta); only the diagonal tile is masked
  const float sc0 = -lse / sl;
  const f32x4 sinit = f32x4{sc0, sc0, sc0, sc0}, dinit = f32x4{-dsum, -dsum, -dsum, -dsum};
  auto tile = [&](const int k0, auto masked) {
    constexpr bool MASK = decltype(masked)::value;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {  // 32 keys: sub-tiles 2 kk and 2 kk + 1
      uint32_t sw[4];
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) {
        const int t = 2 * kk + tt;
        f32x4 sc = sinit, dp = dinit;
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          sc = mfma16(ld16(ks + (16 * t + c) * KLD + 32 * s + 8 * g), qf[s], sc);
          dp = mfma16(ld16(vs + (16 * t + c) * KLD + 32 * s + 8 * g), df[s], dp);
        }
        float d[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float p = __builtin_amdgcn_exp2f(sc[r] * sl);
          if constexpr (MASK) {
            const int key = k0 + 16 * t + 4 * g + r;
            if (!(key <= qi && key < L)) p = 0.f;
          }
          d[r] = p * dp[r];
        }
        sw[2 * tt] = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t{d[0], d[1]}), bf16x2_t));
        sw[2 * tt + 1] = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t{d[2], d[3]}), bf16x2_t));
      }
      const s16x8 sa = __builtin_bit_cast(s16x8, u32x4{sw[0], sw[1], sw[2], sw[3]});
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
        dqT[dt] = mfma16(tr_frag(ks, KLD, kk, dt, g, c), sa, dqT[dt]);
    }
  };

  for (int kt = 0; kt <= qt; ++kt) {
    const int k0 = kt * TT;
    __syncthreads();
    kr.template store<KLD>(ks);
    vr.template store<KLD>(vs);
    __syncthreads();
    if (kt < qt) {
      kr.load(Kb, ldk, k0 + TT, L);
      vr.load(Vb, ldv, k0 + TT, L);
      tile(k0, std::false_type{});  // every key of a tile below the diagonal precedes every query of this one
    } else {
      tile(k0, std::true_type{});
    }
  }
  if (qi >= L) return;
  uint16_t* op = dQ + ((long)b * L + qi) * lddq + h * DH + 4 * g;
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt)
    *reinterpret_cast<s16x4*>(op + 16 * dt) =
        s16x4{(short)f2bf(dqT[dt][0] * scale), (short)f2bf(dqT[dt][1] * scale), (short)f2bf(dqT[dt][2] * scale),
              (short)f2bf(dqT[dt][3] * scale)};
}

template <int DH>
static size_t dkdv_v2_smem() {
  return (size_t)(2 * TT * tr_ld(DH)) * 2 + 2 * TT * sizeof(float);
}

int launch_attn_train_transpose(const uint16_t* x, long ldx, uint16_t* xt, int B, int L, int Lp, int n, int Dh,
                                hipStream_t s) {
  if (B <= 0 || L <= 0) return 0;
  if (Lp % TT != 0 || Lp < L) return -1;
  dim3 grid(Lp / TT, n, B);
  if (Dh == 128)
    attn_train_transpose_kernel<128><<<grid, 256, 0, s>>>(x, ldx, xt, L, Lp, n);
  else if (Dh == 192)
    attn_train_transpose_kernel<192><<<grid, 256, 0, s>>>(x, ldx, xt, L, Lp, n);
  else if (Dh == 64)
    attn_train_transpose_kernel<64><<<grid, 256, 0, s>>>(x, ldx, xt, L, Lp, n);
  else
    return -1;
  return 0;
}

int launch_attn_train_fwd(const uint16_t* q, long ldq, const uint16_t* k, long ldk, const uint16_t* vt, int Lp,
                          uint16_t* o, long ldo, float* lse2, int B, int L, int H, int Hkv, int Dh, float scale,
                          bool causal, hipStream_t s) {
  if (B <= 0 || L <= 0) return 0;
  if (H % Hkv != 0 || Lp % TT != 0 || Lp < L) return -1;
  if (causal && (Dh == 128 || Dh == 64)) {  // v2; the first kernel keeps Dh 192 and the bidirectional case
    const dim3 grid2((L * (H / Hkv) + 255) / 256, Hkv, B);
    const size_t lds = (size_t)3 * 2 * TT * Dh * 2;
    const float sl = scale * L2E;
    if (Dh == 128) {
      static bool attr = hipFuncSetAttribute((const void*)attn_train_fwd_v2_kernel<128>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) == hipSuccess;
      (void)attr;
      attn_train_fwd_v2_kernel<128><<<grid2, 512, lds, s>>>(q, ldq, k, ldk, vt, Lp, o, ldo, lse2, L, H, Hkv, sl);
    } else {
      attn_train_fwd_v2_kernel<64><<<grid2, 512, lds, s>>>(q, ldq, k, ldk, vt, Lp, o, ldo, lse2, L, H, Hkv, sl);
    }
    return 0;
  }
  dim3 grid(H, (L + FQT - 1) / FQT, B);
#define XOT_FWD(DHV, CV) \
  attn_train_fwd_kernel<DHV, CV><<<grid, 256, 0, s>>>(q, ldq, k, ldk, vt, Lp, o, ldo, lse2, L, H, Hkv, scale)
  if (Dh == 192 && causal)
    XOT_FWD(192, true);
  else if (Dh == 128 && causal)
    XOT_FWD(128, true);
  else if (Dh == 128)
    XOT_FWD(128, false);
  else if (Dh == 64 && causal)
    XOT_FWD(64, true);
  else if (Dh == 64)
    XOT_FWD(64, false);
  else
    return -1;
#undef XOT_FWD
  return 0;
}

int launch_attn_train_bwd(const uint16_t* q, long ldq, const uint16_t* k, long ldk, const uint16_t* v, long ldv,
                          const uint16_t* o, long ldo, const uint16_t* dout, long lddo, int Lp, const float* lse2,
                          float* delta, uint16_t* dq, long lddq, uint16_t* dk, long lddk, uint16_t* dv, long lddv,
                          float* ws, long ws_elems, int B, int L, int H, int Hkv, int Dh, float scale, hipStream_t s) {
  if (B <= 0 || L <= 0) return 0;
  if (H % Hkv != 0 || Lp % TT != 0 || Lp < L) return -1;
  const long slab = (long)B * L * Hkv * Dh;
  if (ws == nullptr || ws_elems < 2 * (long)(H / Hkv) * slab) return -1;
  float *wk = ws, *wv = ws + (long)(H / Hkv) * slab;
  // two query heads of a GQA group per dK / dV workgroup (half the fp32 partials; 563 vs 590 us per layer and
  // micro-batch, profiles/r5/train/dkdv_hpw/) when the group size is even
  const int G = H / Hkv, hpw = G % 2 == 0 ? 2 : 1;
  const dim3 gq(H, (L + TT - 1) / TT, B), gk2(H / hpw, (L + DKT - 1) / DKT, B);
#define XOT_BWD(DHV)                                                                                                \
  do {                                                                                                              \
    attn_train_dq_v2_kernel<DHV><<<gq, 256, 0, s>>>(q, ldq, k, ldk, nullptr, v, ldv, o, ldo, dout, lddo, Lp, lse2,   \
                                                    delta, dq, lddq, L, H, Hkv, scale);                             \
    static bool attr2 = hipFuncSetAttribute((const void*)attn_train_dkdv_v2_kernel<DHV>,                           \
                                            hipFuncAttributeMaxDynamicSharedMemorySize,                             \
                                            (int)dkdv_v2_smem<DHV>()) == hipSuccess;                                \
    (void)attr2;                                                                                                    \
    attn_train_dkdv_v2_kernel<DHV><<<gk2, 64 * DKW, dkdv_v2_smem<DHV>(), s>>>(                                      \
        q, ldq, nullptr, k, ldk, v, ldv, dout, lddo, nullptr, Lp, lse2, delta, wk, wv, L, H, Hkv, scale, hpw);      \
  } while (0)
  if (Dh == 128)
    XOT_BWD(128);
  else if (Dh == 192)
    XOT_BWD(192);
  else if (Dh == 64)
    XOT_BWD(64);
  else
    return -1;
#undef XOT_BWD
  const long n4 = slab / 4;
  int blocks = (int)((n4 + 255) / 256);
  if (blocks > 4096) blocks = 4096;
  attn_train_dkdv_reduce_kernel<<<blocks, 256, 0, s>>>(wk, wv, G / hpw, (long)B * L, Hkv * Dh, scale, dk, lddk, dv,
                                                       lddv);
  return 0;
}

}  // namespace xot

// Paged-KV attention for CDNA4 (MFMA 16x16x32 bf16, wave64).
//
// KV cache (one per layer, per shard):  K [num_pages, Hkv, 64, Dh]   V [num_pages, Hkv, 8, Dh, 8]
// V is stored chunk-major inside a page (kernels.h v_page_off): 8 chunks of 8 keys, each chunk [Dh][8], so the
// P.V MFMA operand (8 consecutive keys of one dim) is one 16-B run, a lane group's 16 dims are 256 contiguous
// bytes, and a decode step's new token touches 16 cache lines per KV head (one 16-B run of 8 dims in each)
// instead of the 128 lines of a [Dh][64] transposed page (profiles/r6/headline/v_chunk/).
//
//  decode:  one query token per sequence.  The G = H/Hkv query heads that share a KV head are the
//           16 MFMA rows (GQA packing: K/V are read once per KV head, not once per query head).
//           Split-KV: grid (partitions, Hkv, B); the 4 waves of a workgroup take alternating
//           pages of the partition, keep an online softmax each, and combine through LDS.  A
//           second tiny kernel merges the partitions (log-sum-exp) when there is more than one.
//  prefill: causal, varlen, reads the cache (so chunked prefill / prefix reuse work unchanged).
//           Rows = (new token, head-in-group) pairs, 16 per wave, 64 per workgroup; K and V^T
//           pages are staged through padded LDS (register prefetch of page p+1 under page p).
//
// Softmax runs in the log2 domain (scores pre-multiplied by scale*log2(e), exp2).  Positions and
// the causal mask come from context_lens on device: no mask tensor is ever built or shipped
// (the reference materialises and JSON-ships a [1,T,T] mask per hop, llm_utils.py:473-511).
#include "common.h"
#include "kernels.h"
#include <cstdlib>

namespace xot {

constexpr int PAGE = 64;
constexpr float NEG_BIG = -1e30f;
constexpr float LOG2E = 1.4426950408889634f;

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// ============================================================================ decode
// NW waves share the pages of one (sequence, KV head, partition): 4 (algo 0), or 8 for one partition
// over a short context at small batch (algo 4: at most two pages per wave and no merge launch, where
// each further page a wave walks costs a dependent page-table -> K / V latency of ~3.5 us)
template <int DH, int NW = 4>
__global__ __launch_bounds__(NW * 64) void attn_decode_kernel(
    const uint16_t* __restrict__ q, const uint16_t* __restrict__ kc, const uint16_t* __restrict__ vc,
    const int32_t* __restrict__ block_tables, int max_blocks, const int32_t* __restrict__ ctx_lens,
    uint16_t* __restrict__ out, float* __restrict__ ws_o, float* __restrict__ ws_ml, int H, int Hkv,
    int pages_per_part, int nparts, float scale_log2, int num_pages, int* __restrict__ tickets) {
  constexpr int KS = DH / 32;   // MFMA k-steps over the head dim
  constexpr int NDT = DH / 16;  // 16-wide d tiles of the output
  constexpr int PLD = PAGE + 8;
  __shared__ __attribute__((aligned(16))) uint16_t p_lds[NW][16 * PLD];
  __shared__ float ml_lds[NW][16][2];
  __shared__ float o_lds[NW][16][DH];

  const int part = blockIdx.x, kvh = blockIdx.y, b = blockIdx.z;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, c = lane & 15;
  const int G = H / Hkv;
  const int ctx = min(ctx_lens[b], max_blocks * PAGE);
  const int npages = (ctx + PAGE - 1) / PAGE;
  const int p_begin = part * pages_per_part;
  const int p_end = min(npages, p_begin + pages_per_part);

  // Q fragments (A operand, rows = query heads of this KV group); lane group g owns d in
  // [g*8*KS, (g+1)*8*KS) so every K row read below is one contiguous 16*KS-byte run.
  s16x8 qf[KS];
  {
    const bool ok = c < G;
    const uint16_t* qp = q + ((size_t)b * H + kvh * G + (ok ? c : 0)) * DH + g * 8 * KS;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      s16x8 v = ld16(qp + 8 * s);
      qf[s] = ok ? v : s16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
  }

  float m[4], l[4];
  f32x4 o[NDT];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    m[r] = NEG_BIG;
    l[r] = 0.f;
  }
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int32_t* bt = block_tables + (size_t)b * max_blocks;
  uint16_t* pl = p_lds[wave];
  for (int p = p_begin + wave; p < p_end; p += NW) {
    const long page = min(max(bt[p], 0), num_pages - 1);
    const uint16_t* kb = kc + ((size_t)page * Hkv + kvh) * PAGE * DH;
    const uint16_t* vb = vc + ((size_t)page * Hkv + kvh) * DH * PAGE;
    s16x8 kf[4][KS], vf[NDT][2];
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int s = 0; s < KS; ++s) kf[t][s] = ld16(kb + (16 * t + c) * DH + g * 8 * KS + 8 * s);
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
      for (int k2 = 0; k2 < 2; ++k2) vf[dt][k2] = ld16(vb + v_page_off(8 * (2 * g + k2), 16 * dt + c, DH));

    f32x4 sc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      sc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KS; ++s) sc[t] = mfma16(qf[s], kf[t][s], sc[t]);
    }
    const int key0 = p * PAGE;
    float mt[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) mt[r] = NEG_BIG;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const bool valid = key0 + 16 * t + c < ctx;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        sc[t][r] = valid ? sc[t][r] * scale_log2 : -INFINITY;
        mt[r] = fmaxf(mt[r], sc[t][r]);
      }
    }
    float alpha[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      mt[r] = group16_max(mt[r]);
      const float mn = fmaxf(m[r], mt[r]);
      alpha[r] = exp2f(m[r] - mn);
      m[r] = mn;
      l[r] *= alpha[r];
    }
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float pv = exp2f(sc[t][r] - m[r]);
        l[r] += pv;
        pl[(4 * g + r) * PLD + 16 * t + c] = f2bf(pv);
      }
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
      for (int r = 0; r < 4; ++r) o[dt][r] *= alpha[r];
    wave_lds_sync();
    s16x8 pf[2];
#pragma unroll
    for (int k2 = 0; k2 < 2; ++k2) pf[k2] = ld16(pl + c * PLD + 16 * g + 8 * k2);
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
      for (int k2 = 0; k2 < 2; ++k2) o[dt] = mfma16(pf[k2], vf[dt][k2], o[dt]);
    wave_lds_sync();
  }

  // combine the NW waves (same rows, disjoint pages)
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    l[r] = group16_sum(l[r]);
    if (c == 0) {
      ml_lds[wave][4 * g + r][0] = m[r];
      ml_lds[wave][4 * g + r][1] = l[r];
    }
  }
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
    for (int r = 0; r < 4; ++r) o_lds[wave][4 * g + r][16 * dt + c] = o[dt][r];
  __syncthreads();
  for (int e = threadIdx.x; e < G * DH; e += NW * 64) {
    const int row = e / DH, d = e % DH;
    float M = NEG_BIG;
#pragma unroll
    for (int w = 0; w < NW; ++w) M = fmaxf(M, ml_lds[w][row][0]);
    float L = 0.f, O = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const float f = exp2f(ml_lds[w][row][0] - M);
      L += ml_lds[w][row][1] * f;
      O += o_lds[w][row][d] * f;
    }
    const int h = kvh * G + row;
    if (nparts == 1) {
      out[((size_t)b * H + h) * DH + d] = f2bf(L > 0.f ? O / L : 0.f);
    } else {
      const size_t idx = ((size_t)b * H + h) * nparts + part;
      ws_o[idx * DH + d] = O;
      if (d == 0) {
        ws_ml[idx * 2] = M;
        ws_ml[idx * 2 + 1] = L;
      }
    }
  }
}

template <int DH>
__global__ __launch_bounds__(DH) void attn_decode_reduce_kernel(const float* __restrict__ ws_o,
                                                                const float* __restrict__ ws_ml,
                                                                const int32_t* __restrict__ ctx_lens,
                                                                uint16_t* __restrict__ out, int H, int nparts,
                                                                int pages_per_part) {
  const int bh = blockIdx.x, b = bh / H, d = threadIdx.x;
  const int npages = (max(ctx_lens[b], 0) + PAGE - 1) / PAGE;
  int np = (npages + pages_per_part - 1) / pages_per_part;
  np = np < 1 ? 1 : (np > nparts ? nparts : np);
  const size_t base = (size_t)bh * nparts;
  float M = NEG_BIG;
  for (int p = 0; p < np; ++p) M = fmaxf(M, ws_ml[(base + p) * 2]);
  float L = 0.f, O = 0.f;
  for (int p = 0; p < np; ++p) {
    const float f = exp2f(ws_ml[(base + p) * 2] - M);
    L += ws_ml[(base + p) * 2 + 1] * f;
    O += ws_o[(base + p) * DH + d] * f;
  }
  out[(size_t)bh * DH + d] = f2bf(L > 0.f ? O / L : 0.f);
}

// ---------------------------------------------------------------------------- decode, wave per unit
// One wave owns one (sequence, KV head, KV partition) unit -- no intra-workgroup combine, and units are
// balanced to the page.  Transposed formulation: S^T = K . Q^T (A = 16 keys of K, B = the G query
// heads as columns) so each lane's accumulator column IS one query head: the running max / sum /
// rescale are lane-local scalars, and the probabilities P^T come out of the S^T accumulators already
// in the B-operand layout of O^T += V^T . P^T.  The key held by MFMA row c of score tile t is chosen
// so that this works with contiguous V^T reads: tile t = 2kk + h, row c = 4q + r holds key
// 32kk + 8q + 4h + r, hence lane group g of the P^T operand owns keys 32kk + 8g .. +8 and reads one
// 16-byte run of the transposed V page.  No LDS.
// PF 1: prefetch the next page's K / V into a second register set under the current page's math (378
//       registers: one wave per SIMD).
// PF 2: ONE register set, each half refilled as soon as it is consumed -- the next page's K right after the
//       S^T MFMAs, its V right after the P.V MFMAs -- so a page's loads fly under the other half's math and,
//       at under 256 registers, two waves per SIMD keep twice the pages in flight per CU (algo 5 / 6).
// NT: K / V pages loaded non-temporal (read once per step; algo 3 / 6)
template <int DH, int PF, bool NT>
__device__ __forceinline__ void decode_wave_unit(
    const int unit, const uint16_t* __restrict__ q, const uint16_t* __restrict__ kc, const uint16_t* __restrict__ vc,
    const int32_t* __restrict__ block_tables, int max_blocks, const int32_t* __restrict__ ctx_lens,
    uint16_t* __restrict__ out, float* __restrict__ ws_o, float* __restrict__ ws_ml, int B, int H, int Hkv,
    int pages_per_part, int nparts, float scale_log2, int num_pages, int* __restrict__ tickets, bool vtail) {
  constexpr int KS = DH / 32;   // k-steps of S^T over the head dim
  constexpr int NDT = DH / 16;  // 16-row d tiles of O^T
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4, c = lane & 15;
  const int part = unit % nparts, kvh = (unit / nparts) % Hkv, b = unit / (nparts * Hkv);
  const int G = H / Hkv;
  const int ctx = min(max(ctx_lens[b], 0), max_blocks * PAGE);
  const int npages = (ctx + PAGE - 1) / PAGE;
  const int p_begin = part * pages_per_part;
  const int p_end = min(npages, p_begin + pages_per_part);

  // Q^T (B operand): column c = query head kvh*G + c; k-step s, lane group g: d 32s + 8g .. +8
  // (natural MFMA order, so each K load instruction below reads 64 contiguous bytes of 16 rows).
  s16x8 qf[KS];
  {
    const bool ok = c < G;
    const uint16_t* qp = q + ((size_t)b * H + kvh * G + (ok ? c : 0)) * DH + g * 8;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      s16x8 v = ld16(qp + 32 * s);
      qf[s] = ok ? v : s16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
  }
  float m = NEG_BIG, l = 0.f;
  f32x4 o[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int32_t* bt = block_tables + (size_t)b * max_blocks;
  // K page [64 keys][DH]: score tile t = 2kk + h, lane (g, c) reads key 32kk + 8(c/4) + 4h + c%4,
  //   d 32s + 8g .. +8 for k-step s
  // V page (chunk-major): d tile dt, k-step kk, lane (g, c) reads d 16dt + c, keys 32kk + 8g .. +8 = chunk 4kk + g
  const int krow = 8 * (c >> 2) + (c & 3);
  auto page_of = [&](int p) -> long { return min(max(bt[p], 0), num_pages - 1); };
  auto load_k = [&](int p, long page, s16x8 (&kf)[4][KS]) {
    const uint16_t* kb = kc + ((size_t)page * Hkv + kvh) * PAGE * DH + g * 8;
    // K rows past the context (the tail of the last page) re-read the last valid row: same cache lines,
    // no HBM bytes (their scores are masked).  PMC: the kernel streams HBM at ~6.0 TB/s, and the unused
    // K rows of the last page were ~4 % of its bytes at 525-token contexts.
    const int lim = ctx - 1 - p * PAGE;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int r = min(32 * (t >> 1) + 4 * (t & 1) + krow, lim);
#pragma unroll
      for (int s = 0; s < KS; ++s) kf[t][s] = NT ? ld16nt(kb + r * DH + 32 * s) : ld16(kb + r * DH + 32 * s);
    }
  };
  // Chunks of 8 keys that start past the context (the tail of the last page, vtail) are not read: zeros (their P
  // is 0 anyway, and stale cache contents never reach O).  Lane group g's chunks are 4kk + g, so the skip is per
  // 16-lane group, at 256-B granularity.
  auto load_v = [&](int p, long page, s16x8 (&vf)[NDT][2]) {
    const uint16_t* vb = vc + ((size_t)page * Hkv + kvh) * DH * PAGE + v_page_off(8 * g, c, DH);
    const int left = vtail ? ctx - p * PAGE : PAGE;  // keys of this page inside the context
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      if (8 * (4 * kk + g) < left) {
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) {
          const uint16_t* a = vb + v_page_off(32 * kk, 16 * dt, DH);
          vf[dt][kk] = NT ? ld16nt(a) : ld16(a);
        }
      } else {
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) vf[dt][kk] = s16x8{0, 0, 0, 0, 0, 0, 0, 0};
      }
    }
  };
  auto load = [&](int p, s16x8 (&kf)[4][KS], s16x8 (&vf)[NDT][2]) {
    const long page = page_of(p);
    load_k(p, page, kf);
    load_v(p, page, vf);
  };
  // S^T tiles of page p (consumes K); the rest of the page (softmax, P.V) is pv() below
  auto scores = [&](const s16x8 (&kf)[4][KS], f32x4 (&st)[4]) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      st[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KS; ++s) st[t] = mfma16(kf[t][s], qf[s], st[t]);
    }
  };
  auto pv = [&](int p, f32x4 (&st)[4], const s16x8 (&vf)[NDT][2]) {
    const int key0 = p * PAGE + 8 * g;  // + 32kk + 4h + r
    float mx = NEG_BIG;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = key0 + 32 * (t >> 1) + 4 * (t & 1) + r < ctx ? st[t][r] * scale_log2 : -INFINITY;
        st[t][r] = v;
        mx = fmaxf(mx, v);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float mn = fmaxf(m, mx);
    const float alpha = exp2f(m - mn);
    m = mn;
    l *= alpha;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) o[dt] *= alpha;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      s16x8 pf;
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float pv = exp2f(st[2 * kk + h][r] - mn);
          l += pv;
          pf[4 * h + r] = (short)f2bf(pv);
        }
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) o[dt] = mfma16(vf[dt][kk], pf, o[dt]);
    }
  };
  auto compute = [&](int p, const s16x8 (&kf)[4][KS], const s16x8 (&vf)[NDT][2]) {
    f32x4 st[4];
    scores(kf, st);
    pv(p, st, vf);
  };

  if constexpr (PF == 2) {
    s16x8 kf[4][KS], vf[NDT][2];
    if (p_begin < p_end) load(p_begin, kf, vf);
    for (int p = p_begin; p < p_end; ++p) {
      const bool more = p + 1 < p_end;
      const long nxt = more ? page_of(p + 1) : 0;  // scalar block-table read, ahead of the loads that need it
      f32x4 st[4];
      scores(kf, st);
      if (more) load_k(p + 1, nxt, kf);  // K registers are free once the S^T MFMAs have read them
      pv(p, st, vf);
      if (more) load_v(p + 1, nxt, vf);
    }
  } else if constexpr (PF == 1) {
    s16x8 ka[4][KS], kb2[4][KS];
    s16x8 va[NDT][2], vb2[NDT][2];
    int p = p_begin;
    if (p < p_end) load(p, ka, va);
    for (; p + 1 < p_end; p += 2) {
      load(p + 1, kb2, vb2);
      compute(p, ka, va);
      if (p + 2 < p_end) load(p + 2, ka, va);
      compute(p + 1, kb2, vb2);
    }
    if (p < p_end) compute(p, ka, va);
  } else {
    for (int p = p_begin; p < p_end; ++p) {
      s16x8 kf[4][KS], vf[NDT][2];
      load(p, kf, vf);
      compute(p, kf, vf);
    }
  }

  // lane (g, c): head c, d rows 16dt + 4g + r
  l += __shfl_xor(l, 16, 64);
  l += __shfl_xor(l, 32, 64);
  const int h = kvh * G + c;
  if (nparts == 1) {
    if (c >= G) return;
    const float inv = l > 0.f ? 1.f / l : 0.f;
    uint16_t* op = out + ((size_t)b * H + h) * DH + 4 * g;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
      s16x4 v;
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = (short)f2bf(o[dt][r] * inv);
      *reinterpret_cast<s16x4*>(op + 16 * dt) = v;
    }
    return;
  }
  if (c < G) {
    const size_t idx = ((size_t)b * H + h) * nparts + part;
    float* wo = ws_o + idx * DH + 4 * g;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) *reinterpret_cast<f32x4*>(wo + 16 * dt) = o[dt];
    if (g == 0) {
      ws_ml[idx * 2] = m;
      ws_ml[idx * 2 + 1] = l;
    }
  }
}


// Wave-uniform unit id in an SGPR: page indices and block-table reads stay scalar (s_load, counted by lgkmcnt),
// so they never force a vmcnt(0) drain of the K / V prefetch.  (A strided persistent grid on a subset of the CUs,
// to leave whole CUs to concurrent GEMMs, was measured and dropped: profiles/r4/overlap/.)
template <int DH, int PF, bool NT = false>
__global__ __launch_bounds__(PF == 2 ? 512 : 256, PF == 2 ? 2 : 1) void attn_decode_wave_kernel(
    const uint16_t* __restrict__ q, const uint16_t* __restrict__ kc, const uint16_t* __restrict__ vc,
    const int32_t* __restrict__ block_tables, int max_blocks, const int32_t* __restrict__ ctx_lens,
    uint16_t* __restrict__ out, float* __restrict__ ws_o, float* __restrict__ ws_ml, int B, int H, int Hkv,
    int pages_per_part, int nparts, float scale_log2, int num_pages, int* __restrict__ tickets, int vtail) {
  const int unit = __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
  if (unit >= B * Hkv * nparts) return;  // whole wave
  decode_wave_unit<DH, PF, NT>(unit, q, kc, vc, block_tables, max_blocks, ctx_lens, out, ws_o, ws_ml, B, H, Hkv,
                               pages_per_part, nparts, scale_log2, num_pages, tickets, vtail != 0);
}

int launch_attn_decode(const uint16_t* q, const uint16_t* kc, const uint16_t* vc, const int32_t* block_tables,
                       int max_blocks, const int32_t* ctx_lens, uint16_t* out, float* ws_o, float* ws_ml, int B,
                       int H, int Hkv, int Dh, int pages_per_part, int nparts, float scale, int num_pages, int algo,
                       hipStream_t s, bool merge) {
  // (an in-kernel merge by the last-arriving partition measured slower than the reduce launch in every
  // configuration, profiles/bench_attn_small_r1.json, and was removed in round 6.)  merge = false: the
  // partitions are left in ws_o / ws_ml for the consumer (launch_gemm_stream_merge's prologue at batch 1).
  int* tickets = nullptr;
  const bool reduce = nparts > 1 && merge;
  if (B <= 0) return 0;
  if (H % Hkv != 0 || H / Hkv > 16) return -1;
  dim3 grid(nparts, Hkv, B);
  const float sl = scale * LOG2E;
  if (algo != 0) {  // wave per (sequence, KV head, partition)
    // algo 5 / 6: 8-wave workgroups (two waves per SIMD)
    const int units = B * Hkv * nparts, wpg = algo >= 5 ? 8 : 4;
    const int wgs = (units + wpg - 1) / wpg;
#define XOT_WAVE(DHV, PFV, NTV)                                                                                  \
  attn_decode_wave_kernel<DHV, PFV, NTV><<<wgs, 64 * wpg, 0, s>>>(q, kc, vc, block_tables, max_blocks, ctx_lens, out, ws_o, \
                                                        ws_ml, B, H, Hkv, pages_per_part, nparts, sl, num_pages, tickets, 1)
    // algo 1: no prefetch; 2 / 3: double register set (3: nt loads); 5 / 6: one set refilled per half (6: nt)
    if (Dh == 128) {
      if (algo == 3) XOT_WAVE(128, 1, true); else if (algo == 2) XOT_WAVE(128, 1, false);
      else if (algo == 5) XOT_WAVE(128, 2, false); else if (algo == 6) XOT_WAVE(128, 2, true); else XOT_WAVE(128, 0, false);
      if (reduce) attn_decode_reduce_kernel<128><<<B * H, 128, 0, s>>>(ws_o, ws_ml, ctx_lens, out, H, nparts, pages_per_part);
    } else if (Dh == 64) {
      if (algo == 3) XOT_WAVE(64, 1, true); else if (algo == 2) XOT_WAVE(64, 1, false);
      else if (algo == 5) XOT_WAVE(64, 2, false); else if (algo == 6) XOT_WAVE(64, 2, true); else XOT_WAVE(64, 0, false);
      if (reduce) attn_decode_reduce_kernel<64><<<B * H, 64, 0, s>>>(ws_o, ws_ml, ctx_lens, out, H, nparts, pages_per_part);
    } else {
      return -1;
    }
#undef XOT_WAVE
    return 0;
  }
  if (Dh == 128) {
    attn_decode_kernel<128><<<grid, 256, 0, s>>>(q, kc, vc, block_tables, max_blocks, ctx_lens, out, ws_o, ws_ml,
                                                 H, Hkv, pages_per_part, nparts, sl, num_pages, tickets);
    if (reduce) attn_decode_reduce_kernel<128><<<B * H, 128, 0, s>>>(ws_o, ws_ml, ctx_lens, out, H, nparts, pages_per_part);
  } else if (Dh == 64) {
    attn_decode_kernel<64><<<grid, 256, 0, s>>>(q, kc, vc, block_tables, max_blocks, ctx_lens, out, ws_o, ws_ml, H,
                                                Hkv, pages_per_part, nparts, sl, num_pages, tickets);
    if (reduce) attn_decode_reduce_kernel<64><<<B * H, 64, 0, s>>>(ws_o, ws_ml, ctx_lens, out, H, nparts, pages_per_part);
  } else {
    return -1;
  }
  return 0;
}

void launch_attn_decode_merge(const float* ws_o, const float* ws_ml, const int32_t* ctx_lens, uint16_t* out, int B,
                              int H, int Dh, int nparts, int pages_per_part, hipStream_t s) {
  if (B <= 0) return;
  if (Dh == 128)
    attn_decode_reduce_kernel<128><<<B * H, 128, 0, s>>>(ws_o, ws_ml, ctx_lens, out, H, nparts, pages_per_part);
  else if (Dh == 64)
    attn_decode_reduce_kernel<64><<<B * H, 64, 0, s>>>(ws_o, ws_ml, ctx_lens, out, H, nparts, pages_per_part);
}

// ============================================================================ prefill
template <int DH>
__global__ __launch_bounds__(256) void attn_prefill_kernel(
    const uint16_t* __restrict__ q, const uint16_t* __restrict__ kc, const uint16_t* __restrict__ vc,
    const int32_t* __restrict__ block_tables, int max_blocks, const int32_t* __restrict__ cu_q,
    const int32_t* __restrict__ ctx_lens, uint16_t* __restrict__ out, int H, int Hkv, float scale_log2,
    int num_pages) {
  constexpr int KS = DH / 32, NDT = DH / 16;
  constexpr int KLD = DH + 8, VLD = PAGE + 8, PLD = PAGE + 8;
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  uint16_t* ks = smem;                  // [PAGE][KLD]
  uint16_t* vs = ks + PAGE * KLD;       // [DH][VLD]
  uint16_t* ps = vs + DH * VLD;         // [4][16][PLD]

  const int tile = blockIdx.x, kvh = blockIdx.y, b = blockIdx.z;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c = lane & 15;
  const int G = H / Hkv;
  const int q0 = cu_q[b], qlen = cu_q[b + 1] - q0;
  const int nrows = qlen * G;
  const int row0 = tile * 64;
  if (row0 >= nrows) return;  // whole workgroup exits together
  const int ctx = min(ctx_lens[b], max_blocks * PAGE);
  const int pos0 = ctx - qlen;  // position of the first new token

  // this lane's A-operand row and the 4 C-rows it owns
  const int arow = row0 + 16 * wave + c;
  s16x8 qf[KS];
  {
    const bool ok = arow < nrows;
    const int ti = ok ? arow / G : 0, hi = ok ? arow % G : 0;
    const uint16_t* qp = q + ((size_t)(q0 + ti) * H + kvh * G + hi) * DH + g * 8 * KS;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      s16x8 v = ld16(qp + 8 * s);
      qf[s] = ok ? v : s16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
  }
  int qpos[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int rr = row0 + 16 * wave + 4 * g + r;
    qpos[r] = rr < nrows ? pos0 + rr / G : -1;  // -1: padding row, every key masked
  }
  const int last_row = min(nrows, row0 + 64) - 1;
  const int max_pos = pos0 + last_row / G;
  const int npages = min(max_pos / PAGE + 1, max_blocks);

  float m[4], l[4];
  f32x4 o[NDT];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    m[r] = NEG_BIG;
    l[r] = 0.f;
  }
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int32_t* bt = block_tables + (size_t)b * max_blocks;
  constexpr int CPR = DH / 8;                   // 16-B chunks per K row
  constexpr int NCH = PAGE * DH / 8 / 256;      // chunks per thread per page (K and V each)
  s16x8 rk[NCH], rv[NCH];
  auto gload = [&](int p) {
    const long page = min(max(bt[p], 0), num_pages - 1);
    const uint16_t* kb = kc + ((size_t)page * Hkv + kvh) * PAGE * DH;
    const uint16_t* vb = vc + ((size_t)page * Hkv + kvh) * DH * PAGE;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int qd = tid + 256 * i;
      rk[i] = ld16(kb + qd * 8);
      rv[i] = ld16(vb + qd * 8);
    }
  };
  gload(0);
  uint16_t* pl = ps + wave * 16 * PLD;
  for (int p = 0; p < npages; ++p) {
    __syncthreads();  // previous page fully consumed
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int qd = tid + 256 * i;
      st16(ks + (qd / CPR) * KLD + (qd % CPR) * 8, rk[i]);
      st16(vs + (qd % DH) * VLD + (qd / DH) * 8, rv[i]);  // granule qd = (key chunk qd / DH, dim qd % DH)
    }
    __syncthreads();
    if (p + 1 < npages) gload(p + 1);

    f32x4 sc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      sc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KS; ++s)
        sc[t] = mfma16(qf[s], ld16(ks + (16 * t + c) * KLD + g * 8 * KS + 8 * s), sc[t]);
    }
    const int key0 = p * PAGE;
    float mt[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) mt[r] = NEG_BIG;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int key = key0 + 16 * t + c;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        sc[t][r] = key <= qpos[r] ? sc[t][r] * scale_log2 : -INFINITY;
        mt[r] = fmaxf(mt[r], sc[t][r]);
      }
    }
    float alpha[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      mt[r] = group16_max(mt[r]);
      const float mn = fmaxf(m[r], mt[r]);
      alpha[r] = exp2f(m[r] - mn);
      m[r] = mn;
      l[r] *= alpha[r];
    }
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float pv = exp2f(sc[t][r] - m[r]);
        l[r] += pv;
        pl[(4 * g + r) * PLD + 16 * t + c] = f2bf(pv);
      }
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
      for (int r = 0; r < 4; ++r) o[dt][r] *= alpha[r];
    wave_lds_sync();
    s16x8 pf[2];
#pragma unroll
    for (int k2 = 0; k2 < 2; ++k2) pf[k2] = ld16(pl + c * PLD + 16 * g + 8 * k2);
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
      for (int k2 = 0; k2 < 2; ++k2) o[dt] = mfma16(pf[k2], ld16(vs + (16 * dt + c) * VLD + 16 * g + 8 * k2), o[dt]);
  }

#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float L = group16_sum(l[r]);
    const int rr = row0 + 16 * wave + 4 * g + r;
    if (rr < nrows) {
      const int ti = rr / G, hi = rr % G;
      uint16_t* op = out + ((size_t)(q0 + ti) * H + kvh * G + hi) * DH;
      const float inv = L > 0.f ? 1.f / L : 0.f;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) op[16 * dt + c] = f2bf(o[dt][r] * inv);
    }
  }
}

// ---------------------------------------------------------------------------- prefill v2
// One workgroup = 8 waves = 256 rows (token, head-in-group) of one (sequence, KV head); each wave owns two
// 16-row blocks, so every K / V^T fragment read from LDS feeds two MFMAs.  Transposed formulation as the
// decode wave kernel: S^T = K . Q^T (A = 16 keys of the page, B = Q^T held in registers), so a lane's
// accumulator column is one query row and the online softmax is lane-local except for the two lane-group
// shuffles of the page max; the S^T tile rows take keys in the order 32 kk + 8 (c / 4) + 4 hf + c % 4, so
// the probabilities come out already in the B-operand layout of O^T += V^T . P^T (no LDS round trip for P).
// K and V^T pages (16 KB each at Dh 128) arrive by LDS-DMA into a 2-deep ring, XOR-swizzled per row
// through the per-lane source address (swizzles found by exhaustive search against the ds_read_b128 lane
// groups: every fragment read is conflict-free).  Waves skip the math of pages past their last row's
// position (causal); workgroups are dispatched heaviest tile first, the tiles of one (sequence, KV head)
// kept on one XCD.
template <int DH>
__device__ __forceinline__ int pf_kswz(int r) {
  return DH == 128 ? (3 * (r & 1)) | (((r >> 1) & 1) << 2) | (((r >> 3) & 1) << 3)
                   : (r & 1) | (((r >> 1) & 1) << 1) | (((r >> 3) & 1) << 2);
}

template <int DH>
__global__ __launch_bounds__(512, 1) void attn_prefill_v2_kernel(
    const uint16_t* __restrict__ q, const uint16_t* __restrict__ kc, const uint16_t* __restrict__ vc,
    const int32_t* __restrict__ block_tables, int max_blocks, const int32_t* __restrict__ cu_q,
    const int32_t* __restrict__ ctx_lens, uint16_t* __restrict__ out, int H, int Hkv, float scale_log2,
    int num_pages) {
  constexpr int KS = DH / 32, NDT = DH / 16;
  constexpr int KGPR = DH / 8;                 // 16-B granules per K row
  constexpr int PAGE_EL = PAGE * DH;           // elements of one K (or V^T) page
  constexpr int NCH = 2 * PAGE_EL / 512;       // 1 KB LDS-DMA chunks per page (K then V^T)
  static_assert(NCH % 8 == 0, "chunks split over 8 waves");
  constexpr int CPW = NCH / 8;
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];  // [3][K page | V^T page]

  int tile, kvh, b;
  {
    const int nwg = gridDim.x * gridDim.y * gridDim.z;
    int lin = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    const int xcd = lin & 7, qq = nwg >> 3, rr = nwg & 7;
    lin = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (lin >> 3);
    tile = gridDim.x - 1 - lin % gridDim.x;  // heaviest (latest rows) first
    lin /= gridDim.x;
    kvh = lin % gridDim.y;
    b = lin / gridDim.y;
  }
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c = lane & 15;
  const int G = H / Hkv;
  const int q0 = cu_q[b], qlen = cu_q[b + 1] - q0;
  const int nrows = qlen * G;
  const int row0 = tile * 256;
  if (row0 >= nrows) return;  // whole workgroup exits together
  const int ctx = min(ctx_lens[b], max_blocks * PAGE);
  const int pos0 = ctx - qlen;

  // Q^T fragments (B operand: k = dims, n = rows): lane (g, c) holds row c of block blk, dims 32 s + 8 g .. +8
  s16x8 qf[2][KS];
  int qpos[2];
#pragma unroll
  for (int blk = 0; blk < 2; ++blk) {
    const int row = row0 + 32 * wave + 16 * blk + c;
    const bool ok = row < nrows;
    const int ti = ok ? row / G : 0, hi = ok ? row % G : 0;
    qpos[blk] = ok ? pos0 + ti : -1;
    const uint16_t* qp = q + ((size_t)(q0 + ti) * H + kvh * G + hi) * DH + 8 * g;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const s16x8 v = ld16(qp + 32 * s);
      qf[blk][s] = ok ? v : s16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
  }
  const int last_row = min(nrows, row0 + 256) - 1;
  const int npages = min((pos0 + last_row / G) / PAGE + 1, max_blocks);
  const int wlast = min(nrows - 1, row0 + 32 * wave + 31);
  const int wmax = wlast >= row0 + 32 * wave ? pos0 + wlast / G : -1;  // this wave's last key (causal)
  const int wmin = pos0 + (row0 + 32 * wave) / G;                          // ... and its first row's

  float m[2] = {NEG_BIG, NEG_BIG}, l[2] = {0.f, 0.f};
  f32x4 o[2][NDT];
#pragma unroll
  for (int blk = 0; blk < 2; ++blk)
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) o[blk][dt] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int32_t* bt = block_tables + (size_t)b * max_blocks;
  auto issue = [&](int p, int buf) {
    const long page = min(max(bt[p], 0), num_pages - 1);
    const uint16_t* kb = kc + ((size_t)page * Hkv + kvh) * PAGE_EL;
    const uint16_t* vb = vc + ((size_t)page * Hkv + kvh) * PAGE_EL;
    uint16_t* dst = smem + buf * 2 * PAGE_EL;
#pragma unroll
    for (int i = 0; i < CPW; ++i) {
      const int ch = wave * CPW + i;
      int P = (ch % (NCH / 2)) * 64 + lane;  // granule of the K or V^T image
      const uint16_t* src;
      if (ch < NCH / 2) {
        const int r = P / KGPR, j = (P % KGPR) ^ pf_kswz<DH>(r);
        src = kb + (r * KGPR + j) * 8;
      } else {
        const int r = P >> 3, j = (P & 7) ^ (r & 7);  // V^T image rows: 64 keys = 8 granules (chunks)
        src = vb + v_page_off(8 * j, r, DH);
      }
      __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)(dst + ch * 512), 16, 0, 0);
    }
  };
  // fragment addresses (elements inside a page image), fixed per lane
  int kofs[4][KS];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int r = 32 * (j >> 1) + 8 * (c >> 2) + 4 * (j & 1) + (c & 3);
#pragma unroll
    for (int s = 0; s < KS; ++s) kofs[j][s] = r * DH + 8 * ((4 * s + g) ^ pf_kswz<DH>(r));
  }
  int vofs[2];
  {
    const int r = c;  // V^T row 16 dt + c: (16 dt + c) & 7 == c & 7
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) vofs[kk] = r * PAGE + 8 * ((4 * kk + g) ^ (r & 7));
  }

  // S^T, masking and the online softmax of one page -> P^T fragments and the rescale factors
  auto score = [&](const uint16_t* Ks, int key0, s16x8 (&pf)[2][2], float (&alpha)[2]) {
    f32x4 st[2][4];
#pragma unroll
    for (int blk = 0; blk < 2; ++blk)
#pragma unroll
      for (int j = 0; j < 4; ++j) st[blk][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // K fragments KPF steps ahead of their MFMAs
    constexpr int KPF = 4, NKS = 4 * KS;
    s16x8 ka[KPF];
#pragma unroll
    for (int t = 0; t < KPF - 1; ++t) ka[t] = ld16(Ks + kofs[t & 3][t >> 2]);
#pragma unroll
    for (int t = 0; t < NKS; ++t) {
      if (t + KPF - 1 < NKS) ka[(t + KPF - 1) % KPF] = ld16(Ks + kofs[(t + KPF - 1) & 3][(t + KPF - 1) >> 2]);
      const int j = t & 3, s = t >> 2;
      st[0][j] = mfma16(ka[t % KPF], qf[0][s], st[0][j]);
      st[1][j] = mfma16(ka[t % KPF], qf[1][s], st[1][j]);
      __builtin_amdgcn_sched_barrier(0);
    }
    // softmax on the raw scores: max first (scale > 0 commutes with it), then one fma per score,
    // the bare v_exp_f32 (no denormal range fix-up: the probabilities are rounded to bf16 anyway) and
    // packed bf16 conversions
    const bool need_mask = key0 + PAGE - 1 > wmin;  // wave-uniform
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
      float mt = NEG_BIG;
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) mt = fmaxf(mt, st[blk][j][r]);
      mt = fmaxf(mt, __shfl_xor(mt, 16, 64));
      mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
      const float mn = fmaxf(m[blk], mt * scale_log2);
      alpha[blk] = __builtin_amdgcn_exp2f(m[blk] - mn);
      m[blk] = mn;
      float ls = 0.f;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        u32x4 pw;
#pragma unroll
        for (int e = 0; e < 8; e += 2) {
          const float p0 = __builtin_amdgcn_exp2f(fmaf(st[blk][2 * kk + (e >> 2)][e & 3], scale_log2, -mn));
          const float p1 = __builtin_amdgcn_exp2f(fmaf(st[blk][2 * kk + (e >> 2)][(e & 3) + 1], scale_log2, -mn));
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
    // the running max of a row stops moving after its first pages: skip the rescale when no row of the
    // wave moved (wave-uniform branch)
    if (__ballot(alpha[0] != 1.f || alpha[1] != 1.f)) {
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          o[0][dt][r] *= alpha[0];
          o[1][dt][r] *= alpha[1];
        }
    }
    // V^T fragments VPF dim tiles ahead of their MFMAs (the LDS latency exceeds one tile's 4 MFMAs)
    constexpr int VPF = 3;
    s16x8 va[VPF][2];
#pragma unroll
    for (int t = 0; t < VPF - 1; ++t)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) va[t][kk] = ld16(Vs + vofs[kk] + 16 * t * PAGE);
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
      if (dt + VPF - 1 < NDT) {
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) va[(dt + VPF - 1) % VPF][kk] = ld16(Vs + vofs[kk] + 16 * (dt + VPF - 1) * PAGE);
      }
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        o[0][dt] = mfma16(va[dt % VPF][kk], pf[0][kk], o[0][dt]);
        o[1][dt] = mfma16(va[dt % VPF][kk], pf[1][kk], o[1][dt]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // (Tried: waves 4-7 one page behind on the P.V half, to put one wave's softmax beside its SIMD partner's
  // MFMAs, with a three-page ring -- no faster.)
  // three-page ring, two pages in flight: page p + 2 is issued once every wave is past page p - 1
  if (npages > 0) issue(0, 0);
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
    const int key0 = p * PAGE;
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
    float L = l[blk];
    L += __shfl_xor(L, 16, 64);
    L += __shfl_xor(L, 32, 64);
    const int row = row0 + 32 * wave + 16 * blk + c;
    if (row < nrows) {
      const int ti = row / G, hi = row % G;
      uint16_t* op = out + ((size_t)(q0 + ti) * H + kvh * G + hi) * DH + 4 * g;
      const float inv = L > 0.f ? 1.f / L : 0.f;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
        s16x4 v;
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = (short)f2bf(o[blk][dt][r] * inv);
        *reinterpret_cast<s16x4*>(op + 16 * dt) = v;
      }
    }
  }
}

int launch_attn_prefill(const uint16_t* q, const uint16_t* kc, const uint16_t* vc, const int32_t* block_tables,
                        int max_blocks, const int32_t* cu_q, const int32_t* ctx_lens, uint16_t* out, int B,
                        int max_qlen, int H, int Hkv, int Dh, float scale, int num_pages, int algo, hipStream_t s) {
  if (B <= 0 || max_qlen <= 0) return 0;
  if (H % Hkv != 0) return -1;
  const int G = H / Hkv;
  const float sl = scale * LOG2E;
  if (algo == 2 && (Dh == 128 || Dh == 64)) {
    const dim3 grid2((max_qlen * G + 255) / 256, Hkv, B);
    const size_t lds = (size_t)3 * 2 * 64 * Dh * 2;
    if (Dh == 128) {
      static bool attr = hipFuncSetAttribute((const void*)attn_prefill_v2_kernel<128>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) == hipSuccess;
      (void)attr;
      hipLaunchKernelGGL(attn_prefill_v2_kernel<128>, grid2, dim3(512), lds, s, q, kc, vc, block_tables, max_blocks,
                         cu_q, ctx_lens, out, H, Hkv, sl, num_pages);
    } else {
      hipLaunchKernelGGL(attn_prefill_v2_kernel<64>, grid2, dim3(512), lds, s, q, kc, vc, block_tables, max_blocks,
                         cu_q, ctx_lens, out, H, Hkv, sl, num_pages);
    }
    return 0;
  }
  dim3 grid((max_qlen * G + 63) / 64, Hkv, B);
  if (Dh == 128) {
    const size_t lds = (size_t)(PAGE * (128 + 8) + 128 * (PAGE + 8) + 4 * 16 * (PAGE + 8)) * 2;
    hipLaunchKernelGGL(attn_prefill_kernel<128>, grid, dim3(256), lds, s, q, kc, vc, block_tables, max_blocks, cu_q,
                       ctx_lens, out, H, Hkv, sl, num_pages);
  } else if (Dh == 64) {
    const size_t lds = (size_t)(PAGE * (64 + 8) + 64 * (PAGE + 8) + 4 * 16 * (PAGE + 8)) * 2;
    hipLaunchKernelGGL(attn_prefill_kernel<64>, grid, dim3(256), lds, s, q, kc, vc, block_tables, max_blocks, cu_q,
                       ctx_lens, out, H, Hkv, sl, num_pages);
  } else {
    return -1;
  }
  return 0;
}

}  // namespace xot

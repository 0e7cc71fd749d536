// Paged-KV attention for CDNA4 (MFMA 16x16x32 bf16, wave64).
//
// KV cache (one per layer, per shard):  K [num_pages, Hkv, 64, Dh]   V [num_pages, Hkv, Dh, 64]
// (V is stored transposed inside a page so the P.V MFMA B-operand is contiguous along keys).
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
// Merge the nparts partial (o, m, l) of the G query heads of KV head kvh of sequence b (log-sum-exp).
// Every address depends on the thread's element, so the partials come in by vector loads (the scalar
// cache would bypass the acquire that makes other workgroups' partials visible).
template <int DH>
__device__ __forceinline__ void combine_parts(const float* ws_o, const float* ws_ml, uint16_t* __restrict__ out,
                                              int b, int kvh, int G, int H, int nparts, int tid, int nthr) {
  for (int e = tid; e < G * DH; e += nthr) {
    const int row = e / DH, d = e % DH, h = kvh * G + row;
    const size_t base = ((size_t)b * H + h) * nparts;
    float M = NEG_BIG;
    for (int p = 0; p < nparts; ++p) M = fmaxf(M, ws_ml[(base + p) * 2]);
    float L = 0.f, O = 0.f;
    for (int p = 0; p < nparts; ++p) {
      const float f = exp2f(ws_ml[(base + p) * 2] - M);
      L += ws_ml[(base + p) * 2 + 1] * f;
      O += ws_o[(base + p) * DH + d] * f;
    }
    out[((size_t)b * H + h) * DH + d] = f2bf(L > 0.f ? O / L : 0.f);
  }
}

// Last-arriver hand-off of a partition's partials (cdna_hip_programming.md Guideline 16 recipe): the
// caller's stores are drained, one lane releases at agent scope, drains again, adds to the (sequence,
// KV head) ticket; the last of the nparts arrivals acquires and resets the ticket for the next launch.
__device__ __forceinline__ bool partition_arrive_last(int* tickets, int slot, int nparts) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const int prev = __hip_atomic_fetch_add(tickets + slot, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const bool last = prev == nparts - 1;
  if (last) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(tickets + slot, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  return last;
}

template <int DH>
__global__ __launch_bounds__(256) void attn_decode_kernel(
    const uint16_t* __restrict__ q, const uint16_t* __restrict__ kc, const uint16_t* __restrict__ vc,
    const int32_t* __restrict__ block_tables, int max_blocks, const int32_t* __restrict__ ctx_lens,
    uint16_t* __restrict__ out, float* __restrict__ ws_o, float* __restrict__ ws_ml, int H, int Hkv,
    int pages_per_part, int nparts, float scale_log2, int num_pages, int* __restrict__ tickets) {
  constexpr int KS = DH / 32;   // MFMA k-steps over the head dim
  constexpr int NDT = DH / 16;  // 16-wide d tiles of the output
  constexpr int PLD = PAGE + 8;
  __shared__ __attribute__((aligned(16))) uint16_t p_lds[4][16 * PLD];
  __shared__ float ml_lds[4][16][2];
  __shared__ float o_lds[4][16][DH];

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
  for (int p = p_begin + wave; p < p_end; p += 4) {
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
      for (int k2 = 0; k2 < 2; ++k2) vf[dt][k2] = ld16(vb + (16 * dt + c) * PAGE + 16 * g + 8 * k2);

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

  // combine the 4 waves (same rows, disjoint pages)
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
  for (int e = threadIdx.x; e < G * DH; e += 256) {
    const int row = e / DH, d = e % DH;
    float M = NEG_BIG;
#pragma unroll
    for (int w = 0; w < 4; ++w) M = fmaxf(M, ml_lds[w][row][0]);
    float L = 0.f, O = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
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
  if (nparts > 1 && tickets != nullptr) {  // the last partition of this (sequence, KV head) merges them all
    __shared__ int last_s;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) last_s = partition_arrive_last(tickets, b * Hkv + kvh, nparts);
    __syncthreads();
    if (last_s) combine_parts<DH>(ws_o, ws_ml, out, b, kvh, G, H, nparts, threadIdx.x, 256);
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
// PF: prefetch the next page's K / V into registers under the current page's math.
template <int DH, bool PF>
__global__ __launch_bounds__(256) void attn_decode_wave_kernel(
    const uint16_t* __restrict__ q, const uint16_t* __restrict__ kc, const uint16_t* __restrict__ vc,
    const int32_t* __restrict__ block_tables, int max_blocks, const int32_t* __restrict__ ctx_lens,
    uint16_t* __restrict__ out, float* __restrict__ ws_o, float* __restrict__ ws_ml, int B, int H, int Hkv,
    int pages_per_part, int nparts, float scale_log2, int num_pages, int* __restrict__ tickets) {
  constexpr int KS = DH / 32;   // k-steps of S^T over the head dim
  constexpr int NDT = DH / 16;  // 16-row d tiles of O^T
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4, c = lane & 15;
  // wave-uniform unit id in an SGPR: page indices and block-table reads stay scalar (s_load, counted by
  // lgkmcnt), so they never force a vmcnt(0) drain of the K / V prefetch
  const int unit = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  if (unit >= B * Hkv * nparts) return;  // whole wave
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
  // V^T page [DH][64 keys]: d tile dt, k-step kk, lane (g, c) reads d 16dt + c, keys 32kk + 8g .. +8
  const int krow = 8 * (c >> 2) + (c & 3);
  auto load = [&](int p, s16x8 (&kf)[4][KS], s16x8 (&vf)[NDT][2]) {
    const long page = min(max(bt[p], 0), num_pages - 1);
    const uint16_t* kb = kc + ((size_t)page * Hkv + kvh) * PAGE * DH + g * 8;
    const uint16_t* vb = vc + ((size_t)page * Hkv + kvh) * DH * PAGE + c * PAGE + 8 * g;
    // K rows past the context (the tail of the last page) re-read the last valid row: same cache lines,
    // no HBM bytes (their scores are masked).  PMC: the kernel streams HBM at ~6.0 TB/s, and the unused
    // K rows of the last page were ~4 % of its bytes at 525-token contexts.
    const int lim = ctx - 1 - p * PAGE;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int r = min(32 * (t >> 1) + 4 * (t & 1) + krow, lim);
#pragma unroll
      for (int s = 0; s < KS; ++s) kf[t][s] = ld16(kb + r * DH + 32 * s);
    }
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) vf[dt][kk] = ld16(vb + 16 * dt * PAGE + 32 * kk);
  };
  auto compute = [&](int p, const s16x8 (&kf)[4][KS], const s16x8 (&vf)[NDT][2]) {
    f32x4 st[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      st[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KS; ++s) st[t] = mfma16(kf[t][s], qf[s], st[t]);
    }
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

  if constexpr (PF) {
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
  if (tickets != nullptr) {  // the last partition of this (sequence, KV head) merges them all
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int last = 0;
    if (lane == 0) last = partition_arrive_last(tickets, b * Hkv + kvh, nparts);
    last = __shfl(last, 0, 64);
    // (lane 0's acquire precedes the other lanes' loads: one wave, program order)
    if (last) combine_parts<DH>(ws_o, ws_ml, out, b, kvh, G, H, nparts, lane, 64);
  }
}

int launch_attn_decode(const uint16_t* q, const uint16_t* kc, const uint16_t* vc, const int32_t* block_tables,
                       int max_blocks, const int32_t* ctx_lens, uint16_t* out, float* ws_o, float* ws_ml, int B,
                       int H, int Hkv, int Dh, int pages_per_part, int nparts, float scale, int num_pages, int algo,
                       int* tickets, hipStream_t s) {
  // tickets ([B * Hkv] int32, zero at rest): the last partition merges in-kernel, no reduce launch
  const bool reduce = nparts > 1 && tickets == nullptr;
  if (B <= 0) return 0;
  if (H % Hkv != 0 || H / Hkv > 16) return -1;
  dim3 grid(nparts, Hkv, B);
  const float sl = scale * LOG2E;
  if (algo != 0) {  // wave per (sequence, KV head, partition)
    const int units = B * Hkv * nparts, wgs = (units + 3) / 4;
#define XOT_WAVE(DHV, PFV)                                                                                       \
  attn_decode_wave_kernel<DHV, PFV><<<wgs, 256, 0, s>>>(q, kc, vc, block_tables, max_blocks, ctx_lens, out, ws_o, \
                                                        ws_ml, B, H, Hkv, pages_per_part, nparts, sl, num_pages, tickets)
    if (Dh == 128) {
      if (algo == 2) XOT_WAVE(128, true); else XOT_WAVE(128, false);
      if (reduce) attn_decode_reduce_kernel<128><<<B * H, 128, 0, s>>>(ws_o, ws_ml, ctx_lens, out, H, nparts, pages_per_part);
    } else if (Dh == 64) {
      if (algo == 2) XOT_WAVE(64, true); else XOT_WAVE(64, false);
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
      st16(vs + (qd / (PAGE / 8)) * VLD + (qd % (PAGE / 8)) * 8, rv[i]);
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

int launch_attn_prefill(const uint16_t* q, const uint16_t* kc, const uint16_t* vc, const int32_t* block_tables,
                        int max_blocks, const int32_t* cu_q, const int32_t* ctx_lens, uint16_t* out, int B,
                        int max_qlen, int H, int Hkv, int Dh, float scale, int num_pages, hipStream_t s) {
  if (B <= 0 || max_qlen <= 0) return 0;
  if (H % Hkv != 0) return -1;
  const int G = H / Hkv;
  dim3 grid((max_qlen * G + 63) / 64, Hkv, B);
  const float sl = scale * LOG2E;
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

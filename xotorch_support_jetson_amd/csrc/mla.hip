// DeepSeek multi-head latent attention (MLA) for CDNA4 (MFMA 16x16x32 bf16, wave64).
//
// Cache (one per layer, per shard): C [num_pages, 64, DL + DR] -- per token the normalised kv latent
// (DL = kv_lora_rank) and the rotated shared rope key (DR = qk_rope_head_dim = 64).  576 numbers per
// token for DeepSeek-V2/V3 instead of 2 x heads x 128 (the reference has no MLA at all; HF keeps the
// same latent in its cache, modeling_deepseek_v3.py DeepseekV3Attention).
//
// Absorbed formulation (the key/value up-projections never touch the cache):
//   q_lat[h] = q_nope[h] . W_UK[h]                      (host side: one batched GEMM, [H][T][DL])
//   s[h, j]  = (q_lat[h] . c[j] + q_pe[h] . k_pe[j]) * scale
//   o_lat[h] = softmax_j(s[h, :]) . c[:]                 (this kernel, [H][T][DL])
//   o[h]     = o_lat[h] . W_UV[h]^T                      (host side: batched GEMM)
// so attention is multi-query over one 576-wide key / 512-wide value shared by every head.
//
// Kernel: one workgroup (4 waves) per (query token, 16-head block, KV partition), XCD-aware order.  Each 64-key page is
// copied HBM -> LDS once by LDS-DMA (double-buffered: page p+1 is in flight while page p is consumed) and
// used twice: as K (S^T = K . Q^T, A operand rows = keys read by ds_read_b128, one 16-key tile per wave)
// and as V (O^T += V^T . P^T, A operand = V^T read straight from the row-major image by the gfx950
// transposed LDS read ds_read_b64_tr_b16 -- no transposed copy in HBM or LDS).  The lane column of every
// accumulator is a query head, so the online-softmax max / sum / rescale are lane-local; the page max is
// combined across the 4 waves through LDS, P^T is exchanged through LDS, and each wave owns a quarter of
// the DL output dims.  Decode (one query per sequence) and prefill (causal: a query at position p sees keys
// 0..p) are the same kernel; the query's sequence is found by a binary search over cu_q.
#include "common.h"
#include "kernels.h"

namespace xot {

namespace {
constexpr int PAGE = 64;
constexpr float NEG_BIG = -1e30f;
constexpr float LOG2E = 1.4426950408889634f;

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) void* glb_ptr_t;
typedef __attribute__((address_space(3))) s16x4* lds_s16x4_t;

__device__ __forceinline__ void glds16(const void* g, void* lds_base) {
  __builtin_amdgcn_global_load_lds((glb_ptr_t)g, (lds_ptr_t)lds_base, 16, 0, 0);
}
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// workgroup barrier that does not drain outstanding LDS-DMA (vmcnt) -- those are waited for explicitly
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ s16x4 tr_read(const uint16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t)(p));
}
}  // namespace

// ------------------------------------------------------------------------------------------- prep
// Per token: c = rmsnorm(ckv[:DL]) * kv_ln -> cache[slot][:DL]; k_pe = rope(ckv[DL:]) -> cache[slot][DL:];
// q_pe of every head rotated in place (rotate-half pairs; the loader de-interleaved DeepSeek's pairs).
__global__ __launch_bounds__(256) void mla_prep_kernel(const uint16_t* __restrict__ ckv, long ldc,
                                                       const uint16_t* __restrict__ kv_ln, uint16_t* __restrict__ q,
                                                       long ldq, long qpe_off, const int32_t* __restrict__ pos,
                                                       const float* __restrict__ cos_sin,
                                                       const int64_t* __restrict__ slots, uint16_t* __restrict__ cache,
                                                       int H, int DL, int DR, int max_pos, long nslots, float eps) {
  __shared__ float red[4];
  const int t = blockIdx.x, tid = threadIdx.x;
  const uint16_t* row = ckv + (size_t)t * ldc;
  const int64_t slot = slots[t] < nslots ? slots[t] : -1;
  // rmsnorm of the latent: DL / 8 chunks of 8, at most 256 threads x 1 chunk (DL <= 2048)
  float v[8];
  float ss = 0.f;
  const int nch = DL >> 3;
  if (tid < nch) {
    const s16x8 x = ld16(row + tid * 8);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      v[e] = bf2f(x[e]);
      ss += v[e] * v[e];
    }
  }
  ss = wave_sum(ss);
  if ((tid & 63) == 0) red[tid >> 6] = ss;
  __syncthreads();
  const float inv = rsqrtf((red[0] + red[1] + red[2] + red[3]) / (float)DL + eps);
  if (slot >= 0 && tid < nch) {
    const s16x8 w = ld16(kv_ln + tid * 8);
    s16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (short)f2bf(bf2f(f2bf(v[e] * inv)) * bf2f(w[e]));
    st16(cache + (size_t)slot * (DL + DR) + tid * 8, o);
  }
  int p = pos[t];
  p = p < 0 ? 0 : (p >= max_pos ? max_pos - 1 : p);
  const float* cs = cos_sin + (size_t)p * DR;
  const int half = DR >> 1;
  // rope items: (H + 1) heads x half pairs (the +1 is the shared key)
  for (int w = tid; w < (H + 1) * half; w += 256) {
    const int h = w / half, i = w % half;
    const float c = cs[i], s = cs[half + i];
    if (h < H) {
      uint16_t* x = q + (size_t)t * ldq + qpe_off + (size_t)h * DR;
      const float x0 = bf2f(x[i]), x1 = bf2f(x[i + half]);
      x[i] = f2bf(x0 * c - x1 * s);
      x[i + half] = f2bf(x1 * c + x0 * s);
    } else if (slot >= 0) {
      const uint16_t* x = row + DL;
      const float x0 = bf2f(x[i]), x1 = bf2f(x[i + half]);
      uint16_t* y = cache + (size_t)slot * (DL + DR) + DL;
      y[i] = f2bf(x0 * c - x1 * s);
      y[i + half] = f2bf(x1 * c + x0 * s);
    }
  }
}

void launch_mla_prep(const uint16_t* ckv, long ldc, const uint16_t* kv_ln, uint16_t* q, long ldq, long qpe_off,
                     const int32_t* pos, const float* cos_sin, const int64_t* slots, uint16_t* cache, int T, int H,
                     int DL, int DR, int max_pos, long nslots, float eps, hipStream_t s) {
  if (T <= 0) return;
  mla_prep_kernel<<<T, 256, 0, s>>>(ckv, ldc, kv_ln, q, ldq, qpe_off, pos, cos_sin, slots, cache, H, DL, DR, max_pos,
                                    nslots, eps);
}

// ------------------------------------------------------------------------------------------ attention
template <int DL>
__global__ __launch_bounds__(256, 1) void mla_attn_kernel(
    const uint16_t* __restrict__ q_lat, const uint16_t* __restrict__ q_pe, long ldqpe,
    const uint16_t* __restrict__ cache, const int32_t* __restrict__ block_tables, int max_blocks,
    const int32_t* __restrict__ cu_q, const int32_t* __restrict__ ctx_lens, int B, int T, int H,
    uint16_t* __restrict__ out, float* __restrict__ ws_o, float* __restrict__ ws_ml, int pages_per_part, int nparts,
    float scale_log2, int num_pages) {
  constexpr int DR = 64;
  constexpr int ROW = DL + DR;                   // elements per cached token
  constexpr int KS = ROW / 32;                   // MFMA k-steps of S^T
  constexpr int NCH = PAGE * ROW * 2 / 1024;     // 1 KB LDS-DMA chunks per page
  static_assert(NCH % 4 == 0, "page chunks split over 4 waves");
  constexpr int CPW = NCH / 4;
  constexpr int DW = DL / 4;                     // output dims per wave
  constexpr int NDT = DW / 16;
  constexpr int PLD = PAGE + 8;                  // P^T row stride (keys), padded
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  uint16_t* pbuf = smem + 2 * PAGE * ROW;        // [16 heads][PLD] bf16
  float* red = reinterpret_cast<float*>(pbuf + 16 * PLD);  // [4 waves][16 heads]

  // XCD-aware order: the head blocks of one (token, partition) read the same latent pages, so they get
  // consecutive logical ids that round-robin dispatch places on ONE XCD (one HBM read, the rest from
  // that XCD's L2) instead of spreading them over all 8 L2s (measured 8x the cache bytes from HBM).
  int part, hb, t;
  {
    const int nwg = gridDim.x * gridDim.y * gridDim.z;
    int b = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    const int xcd = b & 7, q = nwg >> 3, r = nwg & 7;
    b = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
    hb = b % gridDim.y;
    b /= gridDim.y;
    part = b % gridDim.x;
    t = b / gridDim.x;
  }
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c = lane & 15;
  const int h = hb * 16 + c;
  const bool hv = h < H;

  // sequence of query token t: largest b with cu_q[b] <= t
  int lo = 0, hi = B - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (cu_q[mid] <= t) lo = mid;
    else hi = mid - 1;
  }
  const int b = lo;
  const int nkeys = min(ctx_lens[b] - (cu_q[b + 1] - 1 - t), max_blocks * PAGE);
  const int npages = nkeys > 0 ? (nkeys + PAGE - 1) / PAGE : 0;
  const int p_begin = part * pages_per_part;
  const int p_end = min(npages, p_begin + pages_per_part);
  const int np = max(0, p_end - p_begin);

  // Q^T fragments (B operand of S^T: k = dims, n = heads): lane (c, g) holds dims 32s + 8g .. +8 of head h
  s16x8 qf[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int d = 32 * s + 8 * g;
    s16x8 x = s16x8{0, 0, 0, 0, 0, 0, 0, 0};
    if (hv) x = d < DL ? ld16(q_lat + ((size_t)h * T + t) * DL + d) : ld16(q_pe + (size_t)t * ldqpe + (size_t)h * DR + (d - DL));
    qf[s] = x;
  }

  float m = NEG_BIG, l = 0.f;  // running max / sum of head c (replicated over the 4 lane groups and waves)
  f32x4 o[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int32_t* bt = block_tables + (size_t)b * max_blocks;
  auto issue = [&](int pi, int buf) {
    const long page = min(max(bt[p_begin + pi], 0), num_pages - 1);
    const uint16_t* src = cache + (size_t)page * PAGE * ROW;
    uint16_t* dst = smem + buf * PAGE * ROW;
#pragma unroll
    for (int i = 0; i < CPW; ++i) {
      const int ch = wave * CPW + i;
      glds16(src + ch * 512 + lane * 8, dst + ch * 512);
    }
  };

  if (np > 0) issue(0, 0);
  for (int pi = 0; pi < np; ++pi) {
    const int buf = pi & 1;
    if (pi + 1 < np) {
      issue(pi + 1, buf ^ 1);
      wait_vm<CPW>();
    } else {
      wait_vm<0>();
    }
    lds_barrier();  // page pi landed for every wave
    const uint16_t* Ks = smem + buf * PAGE * ROW;

    // S^T for this wave's 16 keys: st[r] = S[head c][key 16 wave + 4g + r]
    f32x4 st = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KS; ++s) st = mfma16(ld16(Ks + (16 * wave + c) * ROW + 32 * s + 8 * g), qf[s], st);
    const int key0 = (p_begin + pi) * PAGE + 16 * wave + 4 * g;
    float mt = NEG_BIG;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      st[r] = key0 + r < nkeys ? st[r] * scale_log2 : -INFINITY;
      mt = fmaxf(mt, st[r]);
    }
    mt = fmaxf(mt, __shfl_xor(mt, 16, 64));
    mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
    if (g == 0) red[wave * 16 + c] = mt;
    lds_barrier();
    const float mp = fmaxf(fmaxf(red[c], red[16 + c]), fmaxf(red[32 + c], red[48 + c]));
    const float mn = fmaxf(m, mp);
    const float alpha = exp2f(m - mn);
    m = mn;
    s16x4 pw;
#pragma unroll
    for (int r = 0; r < 4; ++r) pw[r] = (short)f2bf(exp2f(st[r] - m));
    *reinterpret_cast<s16x4*>(pbuf + c * PLD + 16 * wave + 4 * g) = pw;
    lds_barrier();
    // P^T fragments (B operand of O^T: k = keys, n = heads) and the page's row sum of head c
    s16x8 pf[2];
    float ls = 0.f;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      pf[kk] = ld16(pbuf + c * PLD + 32 * kk + 8 * g);
#pragma unroll
      for (int e = 0; e < 8; ++e) ls += bf2f(pf[kk][e]);
    }
    ls += __shfl_xor(ls, 16, 64);
    ls += __shfl_xor(ls, 32, 64);
    l = l * alpha + ls;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
      for (int r = 0; r < 4; ++r) o[dt][r] *= alpha;
    // V^T fragments by transposed LDS reads: lane 4q+p of group g addresses key 32kk + 8g (+4) + q,
    // dims d0 + 4p .. +3; lane c receives dim d0 + c of those 4 keys
    const int q4 = c >> 2, p4 = c & 3;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
      const int d0 = wave * DW + 16 * dt;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const uint16_t* base = Ks + (32 * kk + 8 * g + q4) * ROW + d0 + 4 * p4;
        const s16x4 lo4 = tr_read(base), hi4 = tr_read(base + 4 * ROW);
        const s16x8 vf = s16x8{lo4[0], lo4[1], lo4[2], lo4[3], hi4[0], hi4[1], hi4[2], hi4[3]};
        o[dt] = mfma16(vf, pf[kk], o[dt]);
      }
    }
    lds_barrier();  // every wave is done with this buffer and pbuf before they are refilled
  }

  // o[dt][r] = O[head c][dim wave * DW + 16 dt + 4g + r]
  if (!hv) return;
  if (nparts == 1) {
    const float il = l > 0.f ? 1.f / l : 0.f;
    uint16_t* op = out + ((size_t)h * T + t) * DL + wave * DW + 4 * g;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
      s16x4 v;
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = (short)f2bf(o[dt][r] * il);
      *reinterpret_cast<s16x4*>(op + 16 * dt) = v;
    }
  } else {
    const size_t idx = ((size_t)t * H + h) * nparts + part;
    float* op = ws_o + idx * DL + wave * DW + 4 * g;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) *reinterpret_cast<f32x4*>(op + 16 * dt) = o[dt];
    if (wave == 0 && g == 0) {
      ws_ml[idx * 2] = m;
      ws_ml[idx * 2 + 1] = l;
    }
  }
}

// Many-head variant (DeepSeek-V3 / R1: 128 heads): one workgroup of NW <= 8 waves per (query token, KV
// partition, 16 NW heads).  Every wave owns one 16-head block and does all the page's work for it (S^T of
// all 64 keys, O^T of all DL dims), so a 72 KB page goes HBM -> LDS once for 128 heads instead of once per
// 16-head workgroup (the narrow kernel above: 8x the load traffic, one latency-bound workgroup per CU).
// The four S^T tiles take their K rows in the order key(tile 2kk + hf, row 4g' + r) = 32kk + 8g' + 4hf + r,
// so lane (c, g) ends up with keys 32kk + 8g .. +7 of head c: exactly its P^T B-operand fragment for
// O^T += V^T . P^T -- no LDS exchange, no cross-wave reduction; the page max is two lane shuffles.
template <int DL>
__global__ __launch_bounds__(512, 1) void mla_attn_wide_kernel(
    const uint16_t* __restrict__ q_lat, const uint16_t* __restrict__ q_pe, long ldqpe,
    const uint16_t* __restrict__ cache, const int32_t* __restrict__ block_tables, int max_blocks,
    const int32_t* __restrict__ cu_q, const int32_t* __restrict__ ctx_lens, int B, int T, int H,
    uint16_t* __restrict__ out, float* __restrict__ ws_o, float* __restrict__ ws_ml, int pages_per_part, int nparts,
    float scale_log2, int num_pages) {
  constexpr int DR = 64;
  constexpr int ROW = DL + DR;
  constexpr int KS = ROW / 32;
  constexpr int NCH = PAGE * ROW * 2 / 1024;  // 1 KB LDS-DMA chunks per page
  constexpr int NDT = DL / 16;
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];

  const int nw = blockDim.x >> 6;
  int part, hg, t;
  {  // XCD-aware order (as the narrow kernel): the partitions of one token stay on one XCD
    const int nwg = gridDim.x * gridDim.y * gridDim.z;
    int b = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    const int xcd = b & 7, q = nwg >> 3, r = nwg & 7;
    b = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
    part = b % gridDim.x;
    b /= gridDim.x;
    hg = b % gridDim.y;
    t = b / gridDim.y;
  }
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c = lane & 15;
  const int h = (hg * nw + wave) * 16 + c;
  const bool hv = h < H;

  int lo = 0, hi = B - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (cu_q[mid] <= t) lo = mid;
    else hi = mid - 1;
  }
  const int b = lo;
  const int nkeys = min(ctx_lens[b] - (cu_q[b + 1] - 1 - t), max_blocks * PAGE);
  const int npages = nkeys > 0 ? (nkeys + PAGE - 1) / PAGE : 0;
  const int p_begin = part * pages_per_part;
  const int p_end = min(npages, p_begin + pages_per_part);
  const int np = max(0, p_end - p_begin);

  s16x8 qf[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int d = 32 * s + 8 * g;
    s16x8 x = s16x8{0, 0, 0, 0, 0, 0, 0, 0};
    if (hv) x = d < DL ? ld16(q_lat + ((size_t)h * T + t) * DL + d) : ld16(q_pe + (size_t)t * ldqpe + (size_t)h * DR + (d - DL));
    qf[s] = x;
  }
  float m = NEG_BIG, l = 0.f;
  f32x4 o[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int32_t* bt = block_tables + (size_t)b * max_blocks;
  // LDS image of a page: row r keeps its 16-byte granule j at slot j ^ swz(r) (within its group of 8).  The
  // row stride (ROW * 2 bytes) is an odd multiple of 128 bytes, so the bank half follows the row parity and
  // swz spreads the rest.  swz was found by exhaustive search over XOR maps of the row bits against the
  // ds_read_b128 lane groups ({0-3,12-15,20-27}, {4-11,16-19,28-31}, ...) and the two 32-lane halves of
  // ds_read_b64_tr_b16: both the K row reads (4 LDS cycles) and the transposed V reads (2) are
  // conflict-free (the plain layout: 16 and 8).  LDS-DMA writes linearly, so the permutation is applied
  // through each lane's source address.
  auto swz = [](int r) { return (((r >> 1) & 1) << 1) | (((r >> 3) & 1) << 2); };
  constexpr int GPR = ROW / 8;  // granules per row
  auto issue = [&](int pi, int buf) {
    const long page = min(max(bt[p_begin + pi], 0), num_pages - 1);
    const uint16_t* src = cache + (size_t)page * PAGE * ROW;
    uint16_t* dst = smem + buf * PAGE * ROW;
    for (int ch = wave; ch < NCH; ch += nw) {
      const int P = ch * 64 + lane, r = P / GPR, j = (P - r * GPR) ^ swz(r);
      glds16(src + (r * GPR + j) * 8, dst + ch * 512);
    }
  };
  // K row of S^T tile j (= 2 kk + hf) for MFMA row c: key 32 kk + 8 (c / 4) + 4 hf + c % 4; its k-step s
  // granule 4 s + g sits at slot (4 s + g) ^ swz = 4 (s ^ xb) + xl with x = g ^ swz
  int kb[4][2];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int r = 32 * (j >> 1) + 8 * (c >> 2) + 4 * (j & 1) + (c & 3);
    const int x = g ^ swz(r), xb = x >> 2, xl = x & 3;
    kb[j][0] = r * ROW + 8 * xl + 32 * xb;  // even s: s ^ xb = s + xb
    kb[j][1] = r * ROW + 8 * xl - 32 * xb;  // odd s: s ^ xb = s - xb
  }
  // V^T transposed reads: lane 4 q4 + p4 of group g reads row 32 kk + 8 g + q4 (+4), dims 16 dt + 4 p4 .. +3,
  // i.e. granule 2 dt + p4 / 2 at slot 2 dt ^ y (y = p4 / 2 ^ swz), element 4 (p4 & 1) inside it
  const int q4 = c >> 2, p4 = c & 3;
  int vb[4];
  {
    const int r = 8 * g + q4, y = (p4 >> 1) ^ swz(r), y1 = y >> 1;
#pragma unroll
    for (int v = 0; v < 4; ++v) vb[v] = r * ROW + 16 * (v ^ y1) + 8 * (y & 1) + 4 * (p4 & 1);
  }

  if (np > 0) issue(0, 0);
  for (int pi = 0; pi < np; ++pi) {
    const int buf = pi & 1;
    wait_vm<0>();   // this wave's share of page pi has landed
    lds_barrier();  // ... everyone's, and every wave is done with page pi - 1 (the buffer refilled next)
    if (pi + 1 < np) issue(pi + 1, buf ^ 1);
    const uint16_t* Ks = smem + buf * PAGE * ROW;

    f32x4 st[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) st[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int j = 0; j < 4; ++j) st[j] = mfma16(ld16(Ks + kb[j][s & 1] + 32 * s), qf[s], st[j]);
    const int kbase = (p_begin + pi) * PAGE + 8 * g;
    float mt = NEG_BIG;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = kbase + 32 * (j >> 1) + 4 * (j & 1) + r;
        st[j][r] = key < nkeys ? st[j][r] * scale_log2 : -INFINITY;
        mt = fmaxf(mt, st[j][r]);
      }
    mt = fmaxf(mt, __shfl_xor(mt, 16, 64));
    mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
    const float mn = fmaxf(m, mt);
    const float alpha = exp2f(m - mn);
    m = mn;
    s16x8 pf[2];
    float ls = 0.f;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const uint16_t pb = f2bf(exp2f(st[2 * kk + (e >> 2)][e & 3] - m));
        pf[kk][e] = (short)pb;
        ls += bf2f(pb);
      }
    ls += __shfl_xor(ls, 16, 64);
    ls += __shfl_xor(ls, 32, 64);
    l = l * alpha + ls;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
#pragma unroll
      for (int r = 0; r < 4; ++r) o[dt][r] *= alpha;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const uint16_t* base = Ks + vb[dt & 3] + 32 * kk * ROW + 64 * (dt >> 2);
        const s16x4 lo4 = tr_read(base), hi4 = tr_read(base + 4 * ROW);
        const s16x8 vf = s16x8{lo4[0], lo4[1], lo4[2], lo4[3], hi4[0], hi4[1], hi4[2], hi4[3]};
        o[dt] = mfma16(vf, pf[kk], o[dt]);
      }
    }
  }

  // o[dt][r] = O[head c][dim 16 dt + 4 g + r]
  if (!hv) return;
  if (nparts == 1) {
    const float il = l > 0.f ? 1.f / l : 0.f;
    uint16_t* op = out + ((size_t)h * T + t) * DL + 4 * g;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
      s16x4 v;
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = (short)f2bf(o[dt][r] * il);
      *reinterpret_cast<s16x4*>(op + 16 * dt) = v;
    }
  } else {
    const size_t idx = ((size_t)t * H + h) * nparts + part;
    float* op = ws_o + idx * DL + 4 * g;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) *reinterpret_cast<f32x4*>(op + 16 * dt) = o[dt];
    if (g == 0) {
      ws_ml[idx * 2] = m;
      ws_ml[idx * 2 + 1] = l;
    }
  }
}

// merge the split-KV partials of (token, head): out[h][t][:] = sum_p O_p 2^(m_p - M) / sum_p l_p 2^(m_p - M)
__global__ __launch_bounds__(256) void mla_combine_kernel(const float* __restrict__ ws_o, const float* __restrict__ ws_ml,
                                                          uint16_t* __restrict__ out, int T, int H, int DL, int nparts) {
  const int th = blockIdx.x, t = th / H, h = th % H;
  const size_t base = (size_t)th * nparts;
  float M = NEG_BIG;
  for (int p = 0; p < nparts; ++p) M = fmaxf(M, ws_ml[(base + p) * 2]);
  float L = 0.f;
  for (int p = 0; p < nparts; ++p) L += ws_ml[(base + p) * 2 + 1] * exp2f(ws_ml[(base + p) * 2] - M);
  const float il = L > 0.f ? 1.f / L : 0.f;
  for (int d = threadIdx.x; d < DL; d += 256) {
    float acc = 0.f;
    for (int p = 0; p < nparts; ++p) acc += ws_o[(base + p) * DL + d] * exp2f(ws_ml[(base + p) * 2] - M);
    out[((size_t)h * T + t) * DL + d] = f2bf(acc * il);
  }
}

template <int DL>
static void mla_launch(const uint16_t* q_lat, const uint16_t* q_pe, long ldqpe, const uint16_t* cache,
                       const int32_t* bt, int max_blocks, const int32_t* cu_q, const int32_t* ctx, int B, int T, int H,
                       uint16_t* out, float* ws_o, float* ws_ml, int ppp, int nparts, float scale, int num_pages,
                       int wide, hipStream_t s) {
  constexpr int ROW = DL + 64;
  const int nhb = (H + 15) / 16;
  if (wide) {
    constexpr int SMEM = 2 * PAGE * ROW * 2;
    static_assert(SMEM <= 160 * 1024, "LDS");
    auto kern = mla_attn_wide_kernel<DL>;
    static bool attr = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM) ==
                       hipSuccess;
    (void)attr;
    const int nw = nhb < 8 ? nhb : 8;
    const dim3 grid(nparts, (nhb + nw - 1) / nw, T);
    kern<<<grid, 64 * nw, SMEM, s>>>(q_lat, q_pe, ldqpe, cache, bt, max_blocks, cu_q, ctx, B, T, H, out, ws_o, ws_ml,
                                     ppp, nparts, scale * LOG2E, num_pages);
  } else {
    constexpr int SMEM = 2 * PAGE * ROW * 2 + 16 * (PAGE + 8) * 2 + 4 * 16 * 4;
    static_assert(SMEM <= 160 * 1024, "LDS");
    auto kern = mla_attn_kernel<DL>;
    static bool attr = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM) ==
                       hipSuccess;
    (void)attr;
    const dim3 grid(nparts, nhb, T);
    kern<<<grid, 256, SMEM, s>>>(q_lat, q_pe, ldqpe, cache, bt, max_blocks, cu_q, ctx, B, T, H, out, ws_o, ws_ml, ppp,
                                 nparts, scale * LOG2E, num_pages);
  }
  if (nparts > 1) mla_combine_kernel<<<T * H, 256, 0, s>>>(ws_o, ws_ml, out, T, H, DL, nparts);
}

int launch_mla_attn(const uint16_t* q_lat, const uint16_t* q_pe, long ldqpe, const uint16_t* cache,
                    const int32_t* block_tables, int max_blocks, const int32_t* cu_q, const int32_t* ctx_lens, int B,
                    int T, int H, int DL, int DR, uint16_t* out, float* ws_o, float* ws_ml, int pages_per_part,
                    int nparts, float scale, int num_pages, int wide, hipStream_t s) {
  if (T <= 0) return 0;
  if (DR != 64 || B < 1 || pages_per_part < 1 || nparts < 1) return -1;
  if (nparts > 1 && (ws_o == nullptr || ws_ml == nullptr)) return -1;
  switch (DL) {
    case 512: mla_launch<512>(q_lat, q_pe, ldqpe, cache, block_tables, max_blocks, cu_q, ctx_lens, B, T, H, out, ws_o,
                              ws_ml, pages_per_part, nparts, scale, num_pages, wide, s); return 0;
    case 256: mla_launch<256>(q_lat, q_pe, ldqpe, cache, block_tables, max_blocks, cu_q, ctx_lens, B, T, H, out, ws_o,
                              ws_ml, pages_per_part, nparts, scale, num_pages, wide, s); return 0;
    default: return -1;
  }
}

}  // namespace xot

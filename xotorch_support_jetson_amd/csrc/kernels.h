// Host-side launchers of the gfx950 kernel library (raw pointers + stream; no torch types so the
// kernel translation units compile without the torch headers).  Launchers that can reject a shape
// return -1 and launch nothing; the Python layer turns that into a loud error.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace xot {

void launch_rmsnorm(const uint16_t* x, const uint16_t* res, const uint16_t* w, uint16_t* out, uint16_t* res_out,
                    int rows, int D, float eps, hipStream_t s);
void launch_rmsnorm_bwd(const uint16_t* x, const uint16_t* w, const uint16_t* dy, uint16_t* dx, float* dw,
                        float* dw_part, int rows, int D, float eps, hipStream_t s, const uint16_t* res = nullptr);
int rmsnorm_bwd_part_rows();
void launch_embedding(const int32_t* ids, const uint16_t* table, uint16_t* out, int T, int D, int vocab,
                      hipStream_t s);
void launch_silu_mul(const uint16_t* gu, uint16_t* out, int T, int F, hipStream_t s);
void launch_silu_mul_il(const uint16_t* gu, uint16_t* out, int T, int F, hipStream_t s);
void launch_silu_mul_bwd(const uint16_t* gu, const uint16_t* dout, uint16_t* dgu, int T, int F, hipStream_t s);
void launch_splitk_rope_kv_write(const float* ws, int S, const uint16_t* bias, const int32_t* pos,
                                 const float* cos_sin, const int64_t* slots, uint16_t* q_out, uint16_t* kc,
                                 uint16_t* vc, int T, int H, int Hkv, int Dh, int BS, int max_pos, long nslots,
                                 hipStream_t s);
void launch_rope_kv_write(const uint16_t* qkv, const int32_t* pos, const float* cos_sin, const int64_t* slots,
                          uint16_t* q_out, uint16_t* kc, uint16_t* vc, int T, int H, int Hkv, int Dh, int BS,
                          int max_pos, long nslots, hipStream_t s);
void launch_rope_apply(const uint16_t* x, uint16_t* y, const int32_t* pos, const float* cos_sin, int T, int nh,
                       int Dh, long ldx, long ldy, int max_pos, bool inverse, hipStream_t s);

int launch_gemm_skinny(const uint16_t* X, int ldx, const uint16_t* W, int ldw, const uint16_t* bias,
                       const uint16_t* R, int ldr, void* Y, int ldy, bool out_f32, int epi, int M, int N, int K,
                       int nt, hipStream_t s);
int launch_gemm_stream(const uint16_t* X, int ldx, const uint16_t* W, int ldw, const uint16_t* bias,
                       const uint16_t* R, int ldr, void* Y, int ldy, bool out_f32, int epi, float* ws, long ws_elems,
                       int M, int N, int K, int ntw, int S, bool wshuf, bool reduce, hipStream_t s);
// Batch-1 decode GEMM whose input row is the RMSNorm of a residual projection's pending split-K sum:
// x = rmsnorm(bf16(h + bias + sum_s ws[s])) * lnw, recomputed by every workgroup from the slabs (no separate
// reduce + norm launch); workgroup (0, 0) stores the summed residual row to hout (never h itself: the other
// workgroups are still reading h).  Pre-shuffled bf16 weights, epi none / silu, split-K into ws (a different
// buffer from np.ws).
// The same kernel's other row prologue (launch_gemm_stream_merge): the row is the merge of a batch-1 split-KV
// decode attention's partitions (mo [H][nparts][dh], ml [H][nparts][2], ctx_lens[0]), so the o_proj GEMM replaces
// the attention's merge launch.
struct NormPro {
  const uint16_t* h;
  const float* ws;
  long sstride;
  int S;
  const uint16_t* bias;
  const uint16_t* lnw;
  uint16_t* hout;
  float eps;
  int D;
  const float* mo;
  const float* ml;
  const int32_t* ctx;
  int nparts, ppp, dh;
};
int launch_gemm_stream_merge(const uint16_t* W, float* ws, long ws_elems, int N, int K, int ntw, int S,
                             const NormPro& np, hipStream_t s);
void launch_attn_decode_merge(const float* ws_o, const float* ws_ml, const int32_t* ctx_lens, uint16_t* out, int B,
                              int H, int Dh, int nparts, int pages_per_part, hipStream_t s);
int launch_gemm_stream_norm(const uint16_t* W, const uint16_t* bias, void* Y, int ldy, int epi, float* ws,
                            long ws_elems, int N, int K, int ntw, int S, bool reduce, const NormPro& np,
                            hipStream_t s);
// decode GEMM with weight-only FP8 (e4m3 pre-shuffled tiles + per-row fp32 scale), bf16 activations
int launch_gemm_stream8(const uint16_t* X, int ldx, const uint8_t* W, const float* wscale, const uint16_t* bias,
                        const uint16_t* R, int ldr, void* Y, int ldy, bool out_f32, int epi, float* ws, long ws_elems,
                        int M, int N, int K, int ntw, int S, bool reduce, hipStream_t s);
// large-M GEMM on the pre-shuffled layout (256 x bn x 64 LDS-DMA tiles, 8 waves; split-K via ws)
// four-wave 256 x 256 tile (gemm_w4.hip; tile code 4256 of launch_gemm_big): N % 256 == 0, K % 128 == 0
int launch_gemm_w4(const uint16_t* X, int ldx, const uint16_t* W, const uint16_t* bias, const uint16_t* R, int ldr,
                   void* Y, int ldy, bool out_f32, int epi, float* ws, int M, int N, int K, int S, int group_m,
                   hipStream_t st);
// the same tile on token-major operands (weight gradients): Y [M, N] (+)= Xt^T . Wt, Xt [K, M], Wt [K, N]
int launch_gemm_w4_tn(const uint16_t* Xt, int ldx, const uint16_t* Wt, int ldw, const uint16_t* R, int ldr, void* Y,
                      int ldy, bool out_f32, int epi, int M, int N, int K, int group_m, hipStream_t st);
int gemm_big_group_m();  // grouped raster width of tall grids (XOT_GEMM_GROUP_M)
int launch_gemm_big(const uint16_t* X, int ldx, const uint16_t* W, const uint16_t* bias, const uint16_t* R, int ldr,
                    void* Y, int ldy, bool out_f32, int epi, float* ws, long ws_elems, int M, int N, int K, int bn,
                    int S, bool reduce, hipStream_t s);
// B independent GEMMs Y_e = X_e . W_e^T (pre-shuffled W [B][N][K]; X_e = X + e*xbat, Y_e = Y + e*ybat)
// training-GEMM layouts (csrc/layout.hip): src [R, C] row-major with row stride ld
int launch_shuffle(const uint16_t* src, long ld, uint16_t* dst, int R, int C, hipStream_t s);
int launch_shuffle_t(const uint16_t* src, long ld, uint16_t* dst, int R, int C, hipStream_t s);
int launch_transpose(const uint16_t* src, long ld, uint16_t* dst, int R, int C, hipStream_t s);
int launch_gemm_kgroup(const uint16_t* X, int ldx, const uint16_t* W, uint16_t* Y, int ldy, bool resid,
                       const int* koff, int E, int M, int N, int K, hipStream_t st);
int launch_gemm_batched(const uint16_t* X, int ldx, long xbat, const uint16_t* W, void* Y, int ldy, long ybat,
                        bool out_f32, int B, int M, int N, int K, hipStream_t s);
// h += bias + sum of S fp32 split-K slabs [S][rows][D] (in place, bf16), out = rmsnorm(h) * w
void launch_splitk_resid_rmsnorm(const float* ws, int S, const uint16_t* bias, uint16_t* h, const uint16_t* w,
                                 uint16_t* out, int rows, int D, float eps, hipStream_t s);
// grouped expert GEMM on gemm_big tiles (bm = 128 or 256 rows per tile; large per-expert row counts)
int launch_gemm_moe_big(const uint16_t* X, int ldx, const uint16_t* W, void* Y, int ldy, bool out_f32, int epi,
                        const int* off, const int* gather, int E, int max_rows, int N, int K, int S, long ysplit,
                        int bm, hipStream_t s);
// grouped GEMM over experts: rows of expert e are off[e]..off[e+1] (slot order), W is [E][N][K]
int launch_gemm_moe(const uint16_t* X, int ldx, const uint16_t* W, void* Y, int ldy, bool out_f32, int epi,
                    const int* off, const int* gather, int E, int max_rows, int N, int K, bool wshuf, int S,
                    long ysplit, hipStream_t s);
void launch_splitk_silu(const float* ws, int S, int M, int N, uint16_t* y, hipStream_t s);
int launch_moe_combine_norm(const float* y, const int32_t* slot_of, const float* topw, uint16_t* h,
                            const uint16_t* lnw, uint16_t* out, int T, int k, int D, int S, long ysplit, float eps,
                            hipStream_t s);
int launch_router_logits(const uint16_t* x, const uint16_t* w, float* out, int T, int E, int D, hipStream_t s);
void launch_moe_route(const float* logits, int T, int E, int k, float* topw, int32_t* topi, int32_t* slot_of,
                      int32_t* sorted_tok, int32_t* off, hipStream_t s);
void launch_moe_combine(const float* y, const int32_t* slot_of, const float* topw, uint16_t* h, int T, int k, int D,
                        int S, long ysplit, hipStream_t s);
// DeepSeekMoE routing: method 0 greedy, 1 group max (V2 group_limited_greedy), 2 group top-2 sum (V3 noaux_tc)
// cnt: [E] int32 counters, zero on entry and left zero on exit
int launch_moe_route_ds(const float* logits, const float* bias, int T, int E, int k, int n_group, int topk_group,
                        int method, bool sigmoid, bool norm, float scale, int* cnt, float* topw, int32_t* topi,
                        int32_t* slot_of, int32_t* sorted_tok, int32_t* off, hipStream_t s);
// DeepSeek MLA: latent norm + rope + latent cache write (q_pe rotated in place), and the absorbed attention
void launch_mla_prep(const uint16_t* ckv, long ldc, const uint16_t* kv_ln, uint16_t* q, long ldq, long qpe_off,
                     const int32_t* pos, const float* cos_sin, const int64_t* slots, uint16_t* cache, int T, int H,
                     int DL, int DR, int max_pos, long nslots, float eps, hipStream_t s);
int launch_mla_attn(const uint16_t* q_lat, const uint16_t* q_pe, long ldqpe, const uint16_t* cache,
                    const int32_t* block_tables, int max_blocks, const int32_t* cu_q, const int32_t* ctx_lens, int B,
                    int T, int H, int DL, int DR, uint16_t* out, float* ws_o, float* ws_ml, int pages_per_part,
                    int nparts, float scale, int num_pages, int wide, hipStream_t s);
int launch_gemm_tiled(const uint16_t* X, int ldx, const uint16_t* W, int ldw, const uint16_t* bias,
                      const uint16_t* R, int ldr, void* Y, int ldy, bool out_f32, int epi, int M, int N, int K,
                      hipStream_t s);

int launch_attn_decode(const uint16_t* q, const uint16_t* kc, const uint16_t* vc, const int32_t* block_tables,
                       int max_blocks, const int32_t* ctx_lens, uint16_t* out, float* ws_o, float* ws_ml, int B,
                       int H, int Hkv, int Dh, int pages_per_part, int nparts, float scale, int num_pages, int algo,
                       hipStream_t s, bool merge = true);
int launch_attn_prefill(const uint16_t* q, const uint16_t* kc, const uint16_t* vc, const int32_t* block_tables,
                        int max_blocks, const int32_t* cu_q, const int32_t* ctx_lens, uint16_t* out, int B,
                        int max_qlen, int H, int Hkv, int Dh, float scale, int num_pages, int algo, hipStream_t s);

// causal self-attention for training (token-major Q / K / V slices, GQA); lse2 [B, H, L] fp32 (log2 domain);
// *t arguments are [B, heads, Dh, Lp] transposed images from launch_attn_train_transpose (zero past L)
int launch_attn_train_transpose(const uint16_t* x, long ldx, uint16_t* xt, int B, int L, int Lp, int n, int Dh,
                                hipStream_t s);
int launch_attn_train_fwd(const uint16_t* q, long ldq, const uint16_t* k, long ldk, const uint16_t* vt, int Lp,
                          uint16_t* o, long ldo, float* lse2, int B, int L, int H, int Hkv, int Dh, float scale,
                          bool causal, hipStream_t s);
int launch_attn_train_bwd(const uint16_t* q, long ldq, const uint16_t* k, long ldk, const uint16_t* v, long ldv,
                          const uint16_t* o, long ldo, const uint16_t* dout, long lddo, int Lp, const float* lse2,
                          float* delta, uint16_t* dq, long lddq, uint16_t* dk, long lddk, uint16_t* dv, long lddv,
                          float* ws, long ws_elems, int B, int L, int H, int Hkv, int Dh, float scale, hipStream_t s);

void launch_sample(const float* logits, long ld, int B, int V, const float* temps, int top_k,
                   const int64_t* seed_off, int32_t* out, uint32_t* cand_key, int32_t* cand_idx, hipStream_t s, int algo = -1);
int launch_topk_cand(const float* logits, long ld, int B, int V, int top_k, float* cval, int32_t* cidx, int kc,
                     hipStream_t s);
constexpr int SAMPLE_CAND_PER_ROW = 64 * 64;  // split path scratch: chunks x max top-k

void launch_ce_fwd(const void* x, bool x_f32, long ld, int T, int V, const int32_t* tgt, float* loss, float* lse,
                   hipStream_t s);
void launch_ce_bwd(const void* x, bool x_f32, long ld, int T, int V, const int32_t* tgt, const float* lse,
                   const float* gscale, uint16_t* dx, long ldd, hipStream_t s);
// multi-tensor sum of squares (gradient clipping): batches of up to SUMSQ_MAXT tensors passed by value
constexpr int SUMSQ_MAXT = 64;
struct SumsqBatch {
  const void* p[SUMSQ_MAXT];
  long n[SUMSQ_MAXT];
  int f32[SUMSQ_MAXT];
  int count;
};
int multi_sumsq_chunk();
long multi_sumsq_scratch(int nbatch, int maxc);  // floats of `part`
void launch_multi_sumsq(const SumsqBatch* batches, int nbatch, int maxc, float* part, float* out, hipStream_t s);
int launch_adamw_tiled(float* p, const void* g, bool g_f32, float* m, float* v, uint16_t* pb, uint16_t* ws,
                       uint16_t* wts, int N, int K, float lr, float b1, float b2, float eps, float wd, int step,
                       float gscale, hipStream_t s);
void launch_adamw(float* p, const void* g, bool g_f32, float* m, float* v, uint16_t* p_bf16, long n, float lr,
                  float b1, float b2, float eps, float wd, int step, float gscale, hipStream_t s);

}  // namespace xot

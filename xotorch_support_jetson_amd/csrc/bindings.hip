// Python bindings of the gfx950 kernel library.  Every entry point validates device, dtype,
// contiguity and shapes before launching (a kernel never sees a shape it was not written for);
// outputs are preallocated by the caller so all of these can be captured into a HIP graph.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include "kernels.h"

namespace {

#define XCHECK(cond, ...) TORCH_CHECK(cond, "xot kernel: ", __VA_ARGS__)
#define CHECK_GPU(x) XCHECK((x).is_cuda(), #x " must be a GPU tensor")
#define CHECK_CONTIG(x) XCHECK((x).is_contiguous(), #x " must be contiguous")
#define CHECK_DT(x, dt) XCHECK((x).scalar_type() == (dt), #x " must be " #dt)
#define CHECK_BF16(x) \
  do {                \
    CHECK_GPU(x);     \
    CHECK_DT(x, at::kBFloat16); \
  } while (0)

template <typename... Ts>
bool all_contig_gpu(const Ts&... ts) {
  return ((ts.is_contiguous() && ts.is_cuda()) && ...);
}

inline hipStream_t cur_stream() { return at::hip::getCurrentHIPStream().stream(); }
inline uint16_t* bf(const at::Tensor& t) { return reinterpret_cast<uint16_t*>(t.data_ptr()); }
inline uint16_t* bf_opt(const c10::optional<at::Tensor>& t) {
  return t.has_value() ? reinterpret_cast<uint16_t*>(t->data_ptr()) : nullptr;
}

void rmsnorm(const at::Tensor& x, const at::Tensor& w, at::Tensor& out, const c10::optional<at::Tensor>& res,
             const c10::optional<at::Tensor>& res_out, double eps) {
  CHECK_BF16(x);
  CHECK_BF16(w);
  CHECK_BF16(out);
  CHECK_CONTIG(x);
  CHECK_CONTIG(out);
  const int64_t D = x.size(-1), rows = x.numel() / D;
  XCHECK(D % 8 == 0 && D <= 16384, "rmsnorm: D must be a multiple of 8 and <= 16384");
  XCHECK(w.numel() == D && out.numel() == x.numel(), "rmsnorm: shape mismatch");
  if (res.has_value()) {
    XCHECK(res_out.has_value(), "rmsnorm: residual needs residual_out");
    CHECK_BF16((*res));
    CHECK_BF16((*res_out));
    XCHECK(res->is_contiguous() && res_out->is_contiguous(), "rmsnorm: residual must be contiguous");
    XCHECK(res->numel() == x.numel() && res_out->numel() == x.numel(), "rmsnorm: residual shape mismatch");
  }
  xot::launch_rmsnorm(bf(x), bf_opt(res), bf(w), bf(out), bf_opt(res_out), (int)rows, (int)D, (float)eps,
                      cur_stream());
}

void rmsnorm_bwd(const at::Tensor& x, const at::Tensor& w, const at::Tensor& dy, at::Tensor& dx, at::Tensor& dw,
                 double eps, const c10::optional<at::Tensor>& res) {
  CHECK_BF16(x);
  CHECK_BF16(w);
  CHECK_BF16(dy);
  CHECK_BF16(dx);
  CHECK_GPU(dw);
  CHECK_DT(dw, at::kFloat);
  CHECK_CONTIG(x);
  CHECK_CONTIG(dy);
  CHECK_CONTIG(dx);
  const int64_t D = x.size(-1), rows = x.numel() / D;
  XCHECK(D % 8 == 0 && D <= 16384, "rmsnorm_bwd: bad D");
  XCHECK(dy.numel() == x.numel() && dx.numel() == x.numel() && dw.numel() == D && w.numel() == D,
         "rmsnorm_bwd: shape mismatch");
  if (res.has_value()) {
    CHECK_BF16(*res);
    CHECK_CONTIG(*res);
    XCHECK(res->numel() == x.numel(), "rmsnorm_bwd: res shape");
  }
  const int64_t nblk = (rows + xot::rmsnorm_bwd_part_rows() - 1) / xot::rmsnorm_bwd_part_rows();
  auto part = at::empty({nblk * D}, x.options().dtype(at::kFloat));  // per-block dw partials
  xot::launch_rmsnorm_bwd(bf(x), bf(w), bf(dy), bf(dx), dw.data_ptr<float>(), part.data_ptr<float>(), (int)rows,
                          (int)D, (float)eps, cur_stream(), res.has_value() ? bf(*res) : nullptr);
}

void embedding(const at::Tensor& ids, const at::Tensor& table, at::Tensor& out) {
  CHECK_GPU(ids);
  CHECK_DT(ids, at::kInt);
  CHECK_BF16(table);
  CHECK_BF16(out);
  CHECK_CONTIG(ids);
  CHECK_CONTIG(table);
  CHECK_CONTIG(out);
  const int64_t T = ids.numel(), D = table.size(1);
  XCHECK(D % 8 == 0 && out.numel() == T * D, "embedding: shape mismatch");
  xot::launch_embedding(ids.data_ptr<int32_t>(), bf(table), bf(out), (int)T, (int)D, (int)table.size(0),
                        cur_stream());
}

void silu_mul(const at::Tensor& gu, at::Tensor& out, bool interleaved16) {
  CHECK_BF16(gu);
  CHECK_BF16(out);
  CHECK_CONTIG(gu);
  CHECK_CONTIG(out);
  const int64_t F = out.size(-1), T = out.numel() / F;
  XCHECK(F % 8 == 0 && gu.numel() == 2 * T * F && gu.size(-1) == 2 * F, "silu_mul: shape mismatch");
  if (interleaved16) {
    XCHECK(F % 16 == 0, "silu_mul: interleaved layout needs F % 16 == 0");
    xot::launch_silu_mul_il(bf(gu), bf(out), (int)T, (int)F, cur_stream());
  } else {
    xot::launch_silu_mul(bf(gu), bf(out), (int)T, (int)F, cur_stream());
  }
}

void silu_mul_bwd(const at::Tensor& gu, const at::Tensor& dout, at::Tensor& dgu) {
  CHECK_BF16(gu);
  CHECK_BF16(dout);
  CHECK_BF16(dgu);
  CHECK_CONTIG(gu);
  CHECK_CONTIG(dout);
  CHECK_CONTIG(dgu);
  const int64_t F = dout.size(-1), T = dout.numel() / F;
  XCHECK(F % 8 == 0 && gu.numel() == 2 * T * F && dgu.numel() == gu.numel(), "silu_mul_bwd: shape mismatch");
  xot::launch_silu_mul_bwd(bf(gu), bf(dout), bf(dgu), (int)T, (int)F, cur_stream());
}

void rope_kv_write(const at::Tensor& qkv, const at::Tensor& pos, const at::Tensor& cos_sin, const at::Tensor& slots,
                   at::Tensor& q_out, at::Tensor& k_cache, at::Tensor& v_cache, int64_t H, int64_t Hkv) {
  CHECK_BF16(qkv);
  CHECK_BF16(q_out);
  CHECK_BF16(k_cache);
  CHECK_BF16(v_cache);
  CHECK_GPU(pos);
  CHECK_DT(pos, at::kInt);
  CHECK_GPU(slots);
  CHECK_DT(slots, at::kLong);
  CHECK_GPU(cos_sin);
  CHECK_DT(cos_sin, at::kFloat);
  XCHECK(all_contig_gpu(qkv, pos, cos_sin, slots, q_out), "rope_kv_write: non-contiguous");
  XCHECK(k_cache.is_contiguous() && v_cache.is_contiguous(), "rope_kv_write: cache non-contiguous");
  XCHECK(k_cache.dim() == 4 && v_cache.dim() == 4, "rope_kv_write: caches must be 4-D");
  const int64_t T = pos.numel(), Dh = k_cache.size(3), BS = k_cache.size(2), nb = k_cache.size(0);
  XCHECK(k_cache.size(1) == Hkv && v_cache.size(0) == nb && v_cache.size(1) == Hkv && v_cache.size(2) == Dh &&
             v_cache.size(3) == BS,
         "rope_kv_write: cache layout must be K[nb,Hkv,BS,Dh], V[nb,Hkv,Dh,BS]");
  XCHECK(Dh % 8 == 0 && qkv.numel() == T * (H + 2 * Hkv) * Dh, "rope_kv_write: qkv shape mismatch");
  XCHECK(q_out.numel() == T * H * Dh && slots.numel() == T, "rope_kv_write: q_out/slots shape mismatch");
  XCHECK(cos_sin.dim() == 2 && cos_sin.size(1) == Dh, "rope_kv_write: cos_sin must be [max_pos, Dh]");
  xot::launch_rope_kv_write(bf(qkv), pos.data_ptr<int32_t>(), cos_sin.data_ptr<float>(), slots.data_ptr<int64_t>(),
                            bf(q_out), bf(k_cache), bf(v_cache), (int)T, (int)H, (int)Hkv, (int)Dh, (int)BS,
                            (int)cos_sin.size(0), (long)(nb * BS), cur_stream());
}

void splitk_rope_kv_write(const at::Tensor& ws, int64_t S, const c10::optional<at::Tensor>& bias,
                          const at::Tensor& pos, const at::Tensor& cos_sin, const at::Tensor& slots, at::Tensor& q_out,
                          at::Tensor& k_cache, at::Tensor& v_cache, int64_t H, int64_t Hkv) {
  CHECK_DT(ws, at::kFloat);
  CHECK_BF16(q_out);
  CHECK_BF16(k_cache);
  CHECK_BF16(v_cache);
  CHECK_DT(pos, at::kInt);
  CHECK_DT(slots, at::kLong);
  CHECK_DT(cos_sin, at::kFloat);
  XCHECK(all_contig_gpu(ws, pos, cos_sin, slots, q_out), "splitk_rope_kv_write: non-contiguous");
  XCHECK(k_cache.is_contiguous() && v_cache.is_contiguous() && k_cache.dim() == 4 && v_cache.dim() == 4,
         "splitk_rope_kv_write: caches must be contiguous 4-D");
  const int64_t T = pos.numel(), Dh = k_cache.size(3), BS = k_cache.size(2), nb = k_cache.size(0);
  XCHECK(k_cache.size(1) == Hkv && v_cache.size(0) == nb && v_cache.size(1) == Hkv && v_cache.size(2) == Dh &&
             v_cache.size(3) == BS,
         "splitk_rope_kv_write: cache layout must be K[nb,Hkv,BS,Dh], V[nb,Hkv,Dh,BS]");
  const int64_t N = (H + 2 * Hkv) * Dh;
  XCHECK(Dh % 8 == 0 && S >= 1 && ws.numel() >= S * T * N, "splitk_rope_kv_write: slabs must hold S x T x N");
  XCHECK(q_out.numel() == T * H * Dh && slots.numel() == T, "splitk_rope_kv_write: q_out/slots shape mismatch");
  XCHECK(cos_sin.dim() == 2 && cos_sin.size(1) == Dh, "splitk_rope_kv_write: cos_sin must be [max_pos, Dh]");
  const uint16_t* bp = nullptr;
  if (bias.has_value()) {
    CHECK_BF16((*bias));
    XCHECK(bias->is_contiguous() && bias->numel() == N, "splitk_rope_kv_write: bias shape");
    bp = bf(*bias);
  }
  xot::launch_splitk_rope_kv_write(ws.data_ptr<float>(), (int)S, bp, pos.data_ptr<int32_t>(), cos_sin.data_ptr<float>(),
                                   slots.data_ptr<int64_t>(), bf(q_out), bf(k_cache), bf(v_cache), (int)T, (int)H,
                                   (int)Hkv, (int)Dh, (int)BS, (int)cos_sin.size(0), (long)(nb * BS), cur_stream());
}

void rope_apply(const at::Tensor& x, at::Tensor& y, const at::Tensor& pos, const at::Tensor& cos_sin, int64_t nh,
                int64_t Dh, bool inverse) {
  CHECK_BF16(x);
  CHECK_BF16(y);
  CHECK_GPU(pos);
  CHECK_DT(pos, at::kInt);
  CHECK_DT(cos_sin, at::kFloat);
  XCHECK(x.dim() == 2 && y.dim() == 2 && x.stride(1) == 1 && y.stride(1) == 1, "rope_apply: x/y must be 2-D rows");
  const int64_t T = x.size(0);
  XCHECK(y.size(0) == T && pos.numel() == T && x.size(1) >= nh * Dh && y.size(1) >= nh * Dh && Dh % 8 == 0,
         "rope_apply: shape mismatch");
  XCHECK(cos_sin.dim() == 2 && cos_sin.size(1) == Dh && cos_sin.is_contiguous(), "rope_apply: bad cos_sin");
  xot::launch_rope_apply(bf(x), bf(y), pos.data_ptr<int32_t>(), cos_sin.data_ptr<float>(), (int)T, (int)nh, (int)Dh,
                         x.stride(0), y.stride(0), (int)cos_sin.size(0), inverse, cur_stream());
}

// epi: 0 none, 1 residual add, 2 silu(gate)*up (gate/up interleaved in 16-row tiles)
// algo: 0 auto, 1 skinny, 2 tiled.  nt: n-tiles per wave for the skinny kernel (1 or 2)
void gemm(const at::Tensor& x, const at::Tensor& w, at::Tensor& y, const c10::optional<at::Tensor>& bias,
          const c10::optional<at::Tensor>& res, int64_t epi, int64_t algo, int64_t nt) {
  CHECK_BF16(x);
  CHECK_BF16(w);
  CHECK_GPU(y);
  XCHECK(x.dim() == 2 && w.dim() == 2 && y.dim() == 2, "gemm: x, w, y must be 2-D");
  XCHECK(x.stride(1) == 1 && w.is_contiguous() && y.stride(1) == 1, "gemm: rows must be contiguous");
  const int64_t M = x.size(0), K = x.size(1), N = w.size(0);
  XCHECK(w.size(1) == K, "gemm: K mismatch");
  const bool f32 = y.scalar_type() == at::kFloat;
  XCHECK(f32 || y.scalar_type() == at::kBFloat16, "gemm: y must be bf16 or fp32");
  XCHECK(y.size(0) == M && y.size(1) == (epi == 2 ? N / 2 : N), "gemm: y shape mismatch");
  if (bias.has_value()) {
    CHECK_BF16((*bias));
    XCHECK(bias->numel() == N && bias->is_contiguous(), "gemm: bias shape mismatch");
  }
  int64_t ldr = 0;
  if (epi == 1) {
    XCHECK(res.has_value(), "gemm: residual epilogue needs res");
    CHECK_BF16((*res));
    XCHECK(res->dim() == 2 && res->size(0) == M && res->size(1) == N && res->stride(1) == 1, "gemm: res shape");
    ldr = res->stride(0);
  }
  if (algo == 0) algo = (M <= 128 || epi == 2) ? 1 : 2;
  int rc;
  if (algo == 1)
    rc = xot::launch_gemm_skinny(bf(x), (int)x.stride(0), bf(w), (int)K, bf_opt(bias), epi == 1 ? bf(*res) : nullptr,
                                 (int)ldr, y.data_ptr(), (int)y.stride(0), f32, (int)epi, (int)M, (int)N, (int)K,
                                 (int)nt, cur_stream());
  else
    rc = xot::launch_gemm_tiled(bf(x), (int)x.stride(0), bf(w), (int)K, bf_opt(bias), epi == 1 ? bf(*res) : nullptr,
                                (int)ldr, y.data_ptr(), (int)y.stride(0), f32, (int)epi, (int)M, (int)N, (int)K,
                                cur_stream());
  XCHECK(rc == 0, "gemm: unsupported shape M=", M, " N=", N, " K=", K, " epi=", epi, " algo=", algo);
}

// Decode GEMM v2 (LDS-shared X, streamed W, optional split-K over `splits` workgroup slices with
// an fp32 workspace of >= splits*M*N floats).  ntw: 16-row n-tiles per wave (1 or 2).
void gemm_stream(const at::Tensor& x, const at::Tensor& w, at::Tensor& y, const c10::optional<at::Tensor>& bias,
                 const c10::optional<at::Tensor>& res, const c10::optional<at::Tensor>& ws, int64_t epi, int64_t ntw,
                 int64_t splits, bool wshuf, bool reduce) {
  CHECK_BF16(x);
  CHECK_BF16(w);
  CHECK_GPU(y);
  XCHECK(x.dim() == 2 && w.dim() == 2 && y.dim() == 2, "gemm_stream: x, w, y must be 2-D");
  XCHECK(x.stride(1) == 1 && w.is_contiguous() && y.stride(1) == 1, "gemm_stream: rows must be contiguous");
  // a pre-shuffled weight keeps its logical [N, K] shape (the layout is a permutation of the storage)
  const int64_t M = x.size(0), K = x.size(1), N = w.size(0);
  XCHECK(w.size(1) == K, "gemm_stream: K mismatch");
  const bool f32 = y.scalar_type() == at::kFloat;
  XCHECK(f32 || y.scalar_type() == at::kBFloat16, "gemm_stream: y must be bf16 or fp32");
  XCHECK(y.size(0) == M && y.size(1) == (epi == 2 ? N / 2 : N), "gemm_stream: y shape mismatch");
  XCHECK(M <= 65536, "gemm_stream: M must be <= 65536");
  if (bias.has_value()) {
    CHECK_BF16((*bias));
    XCHECK(bias->numel() == N && bias->is_contiguous(), "gemm_stream: bias shape mismatch");
  }
  int64_t ldr = 0;
  if (epi == 1) {
    XCHECK(res.has_value(), "gemm_stream: residual epilogue needs res");
    CHECK_BF16((*res));
    XCHECK(res->dim() == 2 && res->size(0) == M && res->size(1) == N && res->stride(1) == 1, "gemm_stream: res shape");
    ldr = res->stride(0);
  }
  float* wsp = nullptr;
  long ws_elems = 0;
  if (ws.has_value()) {
    CHECK_GPU((*ws));
    CHECK_DT((*ws), at::kFloat);
    XCHECK(ws->is_contiguous(), "gemm_stream: ws must be contiguous");
    wsp = ws->data_ptr<float>();
    ws_elems = ws->numel();
  }
  if (splits > 1 && epi == 1) XCHECK(res->data_ptr() != nullptr, "gemm_stream: res");
  const int rc = xot::launch_gemm_stream(bf(x), (int)x.stride(0), bf(w), (int)K, bf_opt(bias),
                                         epi == 1 ? bf(*res) : nullptr, (int)ldr, y.data_ptr(), (int)y.stride(0), f32,
                                         (int)epi, wsp, ws_elems, (int)M, (int)N, (int)K, (int)ntw, (int)splits,
                                         wshuf, reduce, cur_stream());
  XCHECK(rc == 0, "gemm_stream: unsupported shape M=", M, " N=", N, " K=", K, " epi=", epi, " ntw=", ntw,
         " splits=", splits);
}

// Batch-1 decode GEMM on pre-shuffled weights whose input row is rmsnorm(bf16(h + bias_in + sum of the S_in slabs of
// ws_in)) * lnw, computed in the GEMM's prologue; the summed residual row is stored to hout (!= h).  y = [1, N] (epi 0)
// or [1, N / 2] (epi 2, SiLU * up); splits > 1 writes fp32 slabs into ws (!= ws_in), reduced unless reduce = false.
void gemm_stream_norm(const at::Tensor& w, at::Tensor& y, const c10::optional<at::Tensor>& bias,
                      const c10::optional<at::Tensor>& ws, int64_t epi, int64_t ntw, int64_t splits, bool reduce,
                      const at::Tensor& h, const c10::optional<at::Tensor>& ws_in, int64_t s_in,
                      const c10::optional<at::Tensor>& bias_in, const at::Tensor& lnw, at::Tensor& hout, double eps) {
  CHECK_BF16(w);
  CHECK_BF16(h);
  CHECK_BF16(lnw);
  CHECK_BF16(hout);
  CHECK_GPU(y);
  XCHECK(w.dim() == 2 && w.is_contiguous(), "gemm_stream_norm: w");
  const int64_t N = w.size(0), K = w.size(1);
  XCHECK(h.dim() == 2 && h.size(0) == 1 && h.size(1) == K && h.is_contiguous(), "gemm_stream_norm: h must be [1, K]");
  XCHECK(hout.sizes() == h.sizes() && hout.is_contiguous() && hout.data_ptr() != h.data_ptr(),
         "gemm_stream_norm: hout must be a distinct [1, K] buffer");
  XCHECK(lnw.numel() == K && lnw.is_contiguous(), "gemm_stream_norm: lnw");
  XCHECK(y.scalar_type() == at::kBFloat16 && y.dim() == 2 && y.size(0) == 1 && y.size(1) == (epi == 2 ? N / 2 : N) &&
             y.stride(1) == 1,
         "gemm_stream_norm: y");
  if (bias.has_value()) {
    CHECK_BF16((*bias));
    XCHECK(bias->numel() == N && bias->is_contiguous(), "gemm_stream_norm: bias");
  }
  if (bias_in.has_value()) {
    CHECK_BF16((*bias_in));
    XCHECK(bias_in->numel() == K && bias_in->is_contiguous(), "gemm_stream_norm: bias_in");
  }
  float* wsp = nullptr;
  long ws_elems = 0;
  if (ws.has_value()) {
    CHECK_GPU((*ws));
    CHECK_DT((*ws), at::kFloat);
    XCHECK(ws->is_contiguous(), "gemm_stream_norm: ws");
    wsp = ws->data_ptr<float>();
    ws_elems = ws->numel();
  }
  xot::NormPro np{bf(h), nullptr, K, (int)s_in, bf_opt(bias_in), bf(lnw), bf(hout), (float)eps, (int)K};
  if (s_in > 0) {
    XCHECK(ws_in.has_value(), "gemm_stream_norm: ws_in");
    CHECK_GPU((*ws_in));
    CHECK_DT((*ws_in), at::kFloat);
    XCHECK(ws_in->is_contiguous() && ws_in->numel() >= s_in * K, "gemm_stream_norm: ws_in holds s_in slabs of K");
    np.ws = ws_in->data_ptr<float>();
  }
  const int rc = xot::launch_gemm_stream_norm(bf(w), bf_opt(bias), y.data_ptr(), (int)y.stride(0), (int)epi, wsp,
                                              ws_elems, (int)N, (int)K, (int)ntw, (int)splits, reduce, np,
                                              cur_stream());
  XCHECK(rc == 0, "gemm_stream_norm: unsupported N=", N, " K=", K, " epi=", epi, " ntw=", ntw, " splits=", splits,
         " s_in=", s_in);
}

// Decode GEMM on FP8 (e4m3) pre-shuffled weights w8 [N, K] uint8 with per-row fp32 scales (y = x . (w8 * s)^T).
void gemm_stream8(const at::Tensor& x, const at::Tensor& w8, const at::Tensor& wscale, at::Tensor& y,
                  const c10::optional<at::Tensor>& bias, const c10::optional<at::Tensor>& res,
                  const c10::optional<at::Tensor>& ws, int64_t epi, int64_t ntw, int64_t splits, bool reduce) {
  CHECK_BF16(x);
  CHECK_GPU(w8);
  CHECK_DT(w8, at::kByte);
  CHECK_GPU(wscale);
  CHECK_DT(wscale, at::kFloat);
  CHECK_GPU(y);
  XCHECK(x.dim() == 2 && w8.dim() == 2 && y.dim() == 2, "gemm_stream8: x, w8, y must be 2-D");
  XCHECK(x.stride(1) == 1 && x.stride(0) % 8 == 0 && w8.is_contiguous() && y.stride(1) == 1 && wscale.is_contiguous(),
         "gemm_stream8: layouts");
  const int64_t M = x.size(0), K = x.size(1), N = w8.size(0);
  XCHECK(w8.size(1) == K && wscale.numel() == N, "gemm_stream8: shapes");
  const bool f32 = y.scalar_type() == at::kFloat;
  XCHECK(f32 || y.scalar_type() == at::kBFloat16, "gemm_stream8: y must be bf16 or fp32");
  XCHECK(y.size(0) == M && y.size(1) == (epi == 2 ? N / 2 : N), "gemm_stream8: y shape");
  if (bias.has_value()) CHECK_BF16((*bias));
  int64_t ldr = 0;
  if (epi == 1) {
    XCHECK(res.has_value(), "gemm_stream8: residual epilogue needs res");
    CHECK_BF16((*res));
    ldr = res->stride(0);
  }
  float* wsp = nullptr;
  long ws_elems = 0;
  if (ws.has_value()) {
    CHECK_GPU((*ws));
    CHECK_DT((*ws), at::kFloat);
    wsp = ws->data_ptr<float>();
    ws_elems = ws->numel();
  }
  const int rc = xot::launch_gemm_stream8(bf(x), (int)x.stride(0), w8.data_ptr<uint8_t>(), wscale.data_ptr<float>(),
                                          bf_opt(bias), epi == 1 ? bf(*res) : nullptr, (int)ldr, y.data_ptr(),
                                          (int)y.stride(0), f32, (int)epi, wsp, ws_elems, (int)M, (int)N, (int)K,
                                          (int)ntw, (int)splits, reduce, cur_stream());
  XCHECK(rc == 0, "gemm_stream8: unsupported shape M=", M, " N=", N, " K=", K, " epi=", epi, " ntw=", ntw,
         " splits=", splits);
}

// Large-M GEMM on the pre-shuffled weight layout (prefill chunks, decode batches > 128 rows).
// bn: 256 or 128 output columns per workgroup; splits > 1 needs an fp32 workspace of splits*M*N.
void gemm_big(const at::Tensor& x, const at::Tensor& w, at::Tensor& y, const c10::optional<at::Tensor>& bias,
              const c10::optional<at::Tensor>& res, const c10::optional<at::Tensor>& ws, int64_t epi, int64_t bn,
              int64_t splits, bool reduce) {
  CHECK_BF16(x);
  CHECK_BF16(w);
  CHECK_GPU(y);
  XCHECK(x.dim() == 2 && w.dim() == 2 && y.dim() == 2, "gemm_big: x, w, y must be 2-D");
  XCHECK(x.stride(1) == 1 && x.stride(0) % 8 == 0 && w.is_contiguous() && y.stride(1) == 1,
         "gemm_big: rows must be contiguous and 16-B aligned");
  const int64_t M = x.size(0), K = x.size(1), N = w.size(0);
  XCHECK(w.size(1) == K, "gemm_big: K mismatch");
  const bool f32 = y.scalar_type() == at::kFloat;
  XCHECK(f32 || y.scalar_type() == at::kBFloat16, "gemm_big: y must be bf16 or fp32");
  XCHECK(y.size(0) == M && y.size(1) == (epi == 2 ? N / 2 : N), "gemm_big: y shape mismatch");
  XCHECK(M <= (1 << 24), "gemm_big: M too large");
  if (bias.has_value()) {
    CHECK_BF16((*bias));
    XCHECK(bias->numel() == N && bias->is_contiguous(), "gemm_big: bias shape mismatch");
  }
  int64_t ldr = 0;
  if (epi == 1) {
    XCHECK(res.has_value(), "gemm_big: residual epilogue needs res");
    CHECK_BF16((*res));
    XCHECK(res->dim() == 2 && res->size(0) == M && res->size(1) == N && res->stride(1) == 1, "gemm_big: res shape");
    ldr = res->stride(0);
  }
  float* wsp = nullptr;
  long ws_elems = 0;
  if (ws.has_value()) {
    CHECK_GPU((*ws));
    CHECK_DT((*ws), at::kFloat);
    XCHECK(ws->is_contiguous(), "gemm_big: ws must be contiguous");
    wsp = ws->data_ptr<float>();
    ws_elems = ws->numel();
  }
  const int rc = xot::launch_gemm_big(bf(x), (int)x.stride(0), bf(w), bf_opt(bias), epi == 1 ? bf(*res) : nullptr,
                                      (int)ldr, y.data_ptr(), (int)y.stride(0), f32, (int)epi, wsp, ws_elems, (int)M,
                                      (int)N, (int)K, (int)bn, (int)splits, reduce, cur_stream());
  XCHECK(rc == 0, "gemm_big: unsupported shape M=", M, " N=", N, " K=", K, " epi=", epi, " bn=", bn,
         " splits=", splits);
}


// B independent projections (MLA's per-head absorbed q . W_UK and o . W_UV^T): y_e = x_e . w_e^T with
// x_e = x.data + e * xbat (rows x.stride(0) apart, K columns), w = [B, N, K] pre-shuffled per problem,
// y_e = y.data + e * ybat (rows ldy apart, N columns).
// Layout kernels of the training GEMMs (csrc/layout.hip).  mode 0: dst = shuffle(src) ([R, C], R % 16,
// C % 128); 1: dst = shuffle(src^T) ([C, R] shuffled; R % 128, C % 64); 2: dst = src^T row-major (same).
void relayout(const at::Tensor& src, at::Tensor& dst, int64_t mode) {
  CHECK_BF16(src);
  CHECK_BF16(dst);
  XCHECK(src.dim() == 2 && src.stride(1) == 1 && src.stride(0) % 8 == 0, "relayout: src must be 2-D with 16-B rows");
  XCHECK(dst.is_contiguous() && dst.numel() == src.numel(), "relayout: dst must be contiguous, same size");
  const int R = (int)src.size(0), C = (int)src.size(1);
  int rc = -1;
  if (mode == 0) rc = xot::launch_shuffle(bf(src), src.stride(0), bf(dst), R, C, cur_stream());
  else if (mode == 1) rc = xot::launch_shuffle_t(bf(src), src.stride(0), bf(dst), R, C, cur_stream());
  else if (mode == 2) rc = xot::launch_transpose(bf(src), src.stride(0), bf(dst), R, C, cur_stream());
  XCHECK(rc == 0, "relayout: unsupported shape R=", R, " C=", C, " mode=", mode);
}

// Weight-gradient GEMM on token-major operands: y [M, N] = dy^T . x (resid: y += dy^T . x, in place), dy [T, M]
// and x [T, N] bf16 with unit column stride (rows may be strided), y bf16 (or fp32 without resid) contiguous.
// M, N multiples of 256, T of 64 (the caller pads ragged token counts with zero rows).
// On the four-wave tile (gemm_w4.hip TN: both operands staged as [64 tokens] row tiles, fragments read transposed).
void gemm_tn(const at::Tensor& dy, const at::Tensor& x, at::Tensor& y, bool resid) {
  CHECK_BF16(dy);
  CHECK_BF16(x);
  CHECK_GPU(y);
  XCHECK(dy.dim() == 2 && x.dim() == 2 && y.dim() == 2, "gemm_tn: 2-D operands");
  XCHECK(dy.stride(1) == 1 && x.stride(1) == 1 && dy.stride(0) % 8 == 0 && x.stride(0) % 8 == 0,
         "gemm_tn: dy / x need unit column stride and 16-B rows");
  const int64_t T = dy.size(0), M = dy.size(1), N = x.size(1);
  XCHECK(x.size(0) == T && y.size(0) == M && y.size(1) == N && y.is_contiguous(), "gemm_tn: shapes");
  const bool f32 = y.scalar_type() == at::kFloat;
  XCHECK(f32 || y.scalar_type() == at::kBFloat16, "gemm_tn: y must be bf16 or fp32");
  XCHECK(!(resid && f32), "gemm_tn: the residual epilogue writes bf16");
  XCHECK(T * std::max(dy.stride(0), x.stride(0)) < (int64_t(1) << 31), "gemm_tn: operands too large");
  const uint16_t* r = resid ? reinterpret_cast<const uint16_t*>(y.data_ptr()) : nullptr;
  const int rc = xot::launch_gemm_w4_tn(bf(dy), (int)dy.stride(0), bf(x), (int)x.stride(0), r, (int)N, y.data_ptr(),
                                        (int)N, f32, resid ? 1 : 0, (int)M, (int)N, (int)T, xot::gemm_big_group_m(),
                                        cur_stream());
  XCHECK(rc == 0, "gemm_tn: unsupported shape M=", M, " N=", N, " T=", T);
}

// K-grouped GEMM (grouped experts' weight gradients): y[e] (+)= x[:, koff[e]:koff[e+1]] . w[:, koff[e]:koff[e+1]]^T,
// x [M, K] row-major bf16, w [N, K] pre-shuffled, y [E, M, N] bf16 contiguous, koff [E+1] int32 (multiples of 64)
void gemm_kgroup(const at::Tensor& x, const at::Tensor& w, at::Tensor& y, const at::Tensor& koff, bool resid) {
  CHECK_BF16(x);
  CHECK_BF16(w);
  CHECK_BF16(y);
  CHECK_GPU(koff);
  CHECK_DT(koff, at::kInt);
  XCHECK(x.dim() == 2 && w.dim() == 2 && y.dim() == 3 && x.stride(1) == 1 && x.stride(0) % 8 == 0, "gemm_kgroup: x");
  XCHECK(w.is_contiguous() && y.is_contiguous() && koff.is_contiguous(), "gemm_kgroup: layout");
  const int64_t M = x.size(0), K = x.size(1), N = w.size(0), E = y.size(0);
  XCHECK(w.size(1) == K && y.size(1) == M && y.size(2) == N && koff.numel() == E + 1, "gemm_kgroup: shapes");
  const int rc = xot::launch_gemm_kgroup(bf(x), (int)x.stride(0), bf(w), bf(y), (int)N, resid, koff.data_ptr<int>(),
                                         (int)E, (int)M, (int)N, (int)K, cur_stream());
  XCHECK(rc == 0, "gemm_kgroup: unsupported shape M=", M, " N=", N, " K=", K);
}

void gemm_batched(const at::Tensor& x, int64_t xbat, int64_t K, const at::Tensor& w, at::Tensor& y, int64_t ybat,
                  int64_t ldy, int64_t M) {
  CHECK_BF16(x);
  CHECK_BF16(w);
  CHECK_GPU(y);
  XCHECK(w.dim() == 3 && w.is_contiguous() && w.size(2) == K, "gemm_batched: w must be [B, N, K] contiguous");
  const int64_t B = w.size(0), N = w.size(1);
  XCHECK(x.stride(-1) == 1 && x.stride(0) % 8 == 0 && xbat % 8 == 0, "gemm_batched: x rows must be 16-B aligned");
  // the last element read, (B-1) xbat + (M-1) ldx + K - 1, must lie inside x's extent
  XCHECK(x.dim() == 2 && x.size(0) >= M && M >= 1 &&
             (B - 1) * xbat + (M - 1) * x.stride(0) + K <= (x.size(0) - 1) * x.stride(0) + x.size(1),
         "gemm_batched: x too small");
  const bool f32 = y.scalar_type() == at::kFloat;
  XCHECK(f32 || y.scalar_type() == at::kBFloat16, "gemm_batched: y must be bf16 or fp32");
  XCHECK(y.is_contiguous() && (B - 1) * ybat + (M - 1) * ldy + N <= y.numel(), "gemm_batched: y too small");
  const int rc = xot::launch_gemm_batched(bf(x), (int)x.stride(0), (long)xbat, bf(w), y.data_ptr(), (int)ldy, (long)ybat,
                                          f32, (int)B, (int)M, (int)N, (int)K, cur_stream());
  XCHECK(rc == 0, "gemm_batched: unsupported shape B=", B, " M=", M, " N=", N, " K=", K);
}

// h [rows, D] += bias + sum_s ws[s] (the split-K slabs of a residual projection, fp32 [S][rows][D]);
// out = rmsnorm(h) * w: the projection's reduce, the residual add and the next RMSNorm in one pass.
void splitk_resid_rmsnorm(const at::Tensor& ws, int64_t splits, const c10::optional<at::Tensor>& bias, at::Tensor& h,
                          const at::Tensor& w, at::Tensor& out, double eps) {
  CHECK_GPU(ws);
  CHECK_DT(ws, at::kFloat);
  CHECK_BF16(h);
  CHECK_BF16(w);
  CHECK_BF16(out);
  XCHECK(all_contig_gpu(ws, h, w, out), "splitk_resid_rmsnorm: tensors must be contiguous GPU");
  const int64_t rows = h.size(0), D = h.size(1);
  XCHECK(h.dim() == 2 && D % 8 == 0 && w.numel() == D && out.numel() == rows * D, "splitk_resid_rmsnorm: shapes");
  XCHECK(splits >= 1 && ws.numel() >= splits * rows * D, "splitk_resid_rmsnorm: workspace too small");
  if (bias.has_value()) {
    CHECK_BF16((*bias));
    XCHECK(bias->numel() == D && bias->is_contiguous(), "splitk_resid_rmsnorm: bias");
  }
  xot::launch_splitk_resid_rmsnorm(ws.data_ptr<float>(), (int)splits, bf_opt(bias), bf(h), bf(w), bf(out), (int)rows,
                                   (int)D, (float)eps, cur_stream());
}

// grouped expert GEMM: y[slot] = x[gather ? gather[slot] : slot] @ w[e].T for slots of expert e
// splits > 1 (fp32 output, no epilogue): K slice s writes rows [s*slots, (s+1)*slots) of y ([splits*slots, N]),
// summed by moe_combine(..., splits)
// big_bm = 128 / 256: gemm_big tiles (pre-shuffled weights), else the weight-streaming kernel
void gemm_moe(const at::Tensor& x, const at::Tensor& w, at::Tensor& y, const at::Tensor& off,
              const c10::optional<at::Tensor>& gather, int64_t epi, int64_t max_rows, bool wshuf, int64_t splits,
              int64_t big_bm) {
  CHECK_BF16(x);
  CHECK_BF16(w);
  CHECK_GPU(y);
  CHECK_GPU(off);
  CHECK_DT(off, at::kInt);
  XCHECK(x.dim() == 2 && w.dim() == 3 && y.dim() == 2, "gemm_moe: x [rows, K], w [E, N, K], y [slots, N']");
  XCHECK(x.stride(1) == 1 && w.is_contiguous() && y.is_contiguous() && off.is_contiguous(), "gemm_moe: layout");
  const int64_t E = w.size(0), N = w.size(1), K = w.size(2);
  XCHECK(x.size(1) == K, "gemm_moe: K mismatch");
  XCHECK(off.numel() == E + 1, "gemm_moe: off must have E+1 entries");
  XCHECK(epi == 0 || epi == 2, "gemm_moe: epilogue must be none or silu");
  const bool f32 = y.scalar_type() == at::kFloat;
  XCHECK(f32 || y.scalar_type() == at::kBFloat16, "gemm_moe: y must be bf16 or fp32");
  XCHECK(y.size(1) == (epi == 2 ? N / 2 : N), "gemm_moe: y width mismatch");
  XCHECK(splits >= 1 && y.size(0) % splits == 0, "gemm_moe: y rows must be splits * slots");
  const int64_t slots = y.size(0) / splits;
  XCHECK(max_rows >= 0 && max_rows <= slots, "gemm_moe: max_rows must be <= slots");
  const int* gp = nullptr;
  if (gather.has_value()) {
    CHECK_GPU((*gather));
    CHECK_DT((*gather), at::kInt);
    XCHECK(gather->is_contiguous() && gather->numel() == slots, "gemm_moe: gather must have one entry per slot");
    gp = gather->data_ptr<int>();
  } else {
    XCHECK(x.size(0) == slots, "gemm_moe: without gather, x rows are slots");
  }
  int rc;
  if (big_bm > 0) {
    XCHECK(wshuf, "gemm_moe: the big-tile path needs pre-shuffled expert weights");
    rc = xot::launch_gemm_moe_big(bf(x), (int)x.stride(0), bf(w), y.data_ptr(), (int)y.stride(0), f32, (int)epi,
                                  off.data_ptr<int>(), gp, (int)E, (int)max_rows, (int)N, (int)K, (int)splits,
                                  (long)(slots * y.size(1)), (int)big_bm, cur_stream());
  } else {
    rc = xot::launch_gemm_moe(bf(x), (int)x.stride(0), bf(w), y.data_ptr(), (int)y.stride(0), f32, (int)epi,
                              off.data_ptr<int>(), gp, (int)E, (int)max_rows, (int)N, (int)K, wshuf, (int)splits,
                              (long)(slots * y.size(1)), cur_stream());
  }
  XCHECK(rc == 0, "gemm_moe: unsupported shape N=", N, " K=", K, " epi=", epi, " splits=", splits);
}

void router_logits(const at::Tensor& x, const at::Tensor& w, at::Tensor& out) {
  CHECK_BF16(x);
  CHECK_BF16(w);
  CHECK_DT(out, at::kFloat);
  XCHECK(all_contig_gpu(x, w, out) && x.dim() == 2 && w.dim() == 2 && out.dim() == 2, "router_logits: 2-D contiguous");
  const int64_t T = x.size(0), D = x.size(1), E = w.size(0);
  XCHECK(w.size(1) == D && out.size(0) == T && out.size(1) == E, "router_logits: shape mismatch");
  const int rc = xot::launch_router_logits(bf(x), bf(w), out.data_ptr<float>(), (int)T, (int)E, (int)D, cur_stream());
  XCHECK(rc == 0, "router_logits: unsupported E=", E, " D=", D);
}

void moe_route(const at::Tensor& logits, int64_t k, at::Tensor& topw, at::Tensor& topi, at::Tensor& slot_of,
               at::Tensor& sorted_tok, at::Tensor& off) {
  CHECK_GPU(logits);
  CHECK_DT(logits, at::kFloat);
  XCHECK(all_contig_gpu(logits, topw, topi, slot_of, sorted_tok, off), "moe_route: tensors must be contiguous GPU");
  const int64_t T = logits.size(0), E = logits.size(1);
  XCHECK(E >= 1 && E <= 64 && k >= 1 && k <= 8 && k <= E, "moe_route: need 1 <= k <= E <= 64, k <= 8");
  CHECK_DT(topw, at::kFloat);
  CHECK_DT(topi, at::kInt);
  CHECK_DT(slot_of, at::kInt);
  CHECK_DT(sorted_tok, at::kInt);
  CHECK_DT(off, at::kInt);
  XCHECK(topw.numel() == T * k && topi.numel() == T * k && slot_of.numel() == T * k && sorted_tok.numel() == T * k &&
             off.numel() == E + 1,
         "moe_route: output sizes");
  xot::launch_moe_route(logits.data_ptr<float>(), (int)T, (int)E, (int)k, topw.data_ptr<float>(), topi.data_ptr<int>(),
                        slot_of.data_ptr<int>(), sorted_tok.data_ptr<int>(), off.data_ptr<int>(), cur_stream());
}

void moe_route_ds(const at::Tensor& logits, const c10::optional<at::Tensor>& bias, int64_t k, int64_t n_group,
                  int64_t topk_group, int64_t method, bool sigmoid, bool norm, double scale, at::Tensor& cnt,
                  at::Tensor& topw, at::Tensor& topi, at::Tensor& slot_of, at::Tensor& sorted_tok, at::Tensor& off) {
  CHECK_GPU(logits);
  CHECK_DT(logits, at::kFloat);
  CHECK_DT(cnt, at::kInt);
  XCHECK(all_contig_gpu(logits, cnt, topw, topi, slot_of, sorted_tok, off), "moe_route_ds: tensors must be contiguous GPU");
  XCHECK(cnt.numel() >= logits.size(1), "moe_route_ds: cnt needs one (zeroed) counter per expert");
  const int64_t T = logits.size(0), E = logits.size(1);
  if (bias.has_value()) {
    CHECK_DT((*bias), at::kFloat);
    XCHECK(bias->is_cuda() && bias->is_contiguous() && bias->numel() == E, "moe_route_ds: bias [E] fp32");
  }
  CHECK_DT(topw, at::kFloat);
  CHECK_DT(topi, at::kInt);
  CHECK_DT(slot_of, at::kInt);
  CHECK_DT(sorted_tok, at::kInt);
  CHECK_DT(off, at::kInt);
  XCHECK(topw.numel() == T * k && topi.numel() == T * k && slot_of.numel() == T * k && sorted_tok.numel() == T * k &&
             off.numel() == E + 1,
         "moe_route_ds: output sizes");
  const int rc = xot::launch_moe_route_ds(logits.data_ptr<float>(), bias.has_value() ? bias->data_ptr<float>() : nullptr,
                                          (int)T, (int)E, (int)k, (int)n_group, (int)topk_group, (int)method, sigmoid,
                                          norm, (float)scale, cnt.data_ptr<int>(), topw.data_ptr<float>(), topi.data_ptr<int>(),
                                          slot_of.data_ptr<int>(), sorted_tok.data_ptr<int>(), off.data_ptr<int>(),
                                          cur_stream());
  XCHECK(rc == 0, "moe_route_ds: unsupported E=", E, " k=", k, " groups=", n_group, "/", topk_group);
}

// ckv [T, >= DL + DR] (row stride ldc), q [T, ldq] with q_pe of head h at qpe_off + h * DR (rotated in place)
void mla_prep(const at::Tensor& ckv, const at::Tensor& kv_ln, at::Tensor& q, int64_t qpe_off, int64_t H,
              const at::Tensor& pos, const at::Tensor& cos_sin, const at::Tensor& slots, at::Tensor& cache, double eps) {
  CHECK_BF16(ckv);
  CHECK_BF16(kv_ln);
  CHECK_BF16(q);
  CHECK_BF16(cache);
  CHECK_DT(pos, at::kInt);
  CHECK_DT(cos_sin, at::kFloat);
  CHECK_DT(slots, at::kLong);
  XCHECK(all_contig_gpu(kv_ln, pos, cos_sin, slots, cache), "mla_prep: contiguous GPU tensors");
  XCHECK(ckv.dim() == 2 && ckv.stride(1) == 1 && q.dim() == 2 && q.stride(1) == 1, "mla_prep: row-major 2-D ckv / q");
  const int64_t T = ckv.size(0), DL = kv_ln.numel(), DR = cos_sin.size(1);
  XCHECK(cache.dim() == 3 && cache.size(1) == 64 && cache.size(2) == DL + DR, "mla_prep: cache [pages, 64, DL + DR]");
  XCHECK(DL % 8 == 0 && DL <= 2048 && DR % 2 == 0 && ckv.size(1) >= DL + DR, "mla_prep: latent / rope dims");
  XCHECK(q.size(0) == T && pos.numel() == T && slots.numel() == T && qpe_off + H * DR <= q.size(1), "mla_prep: shapes");
  xot::launch_mla_prep(bf(ckv), (long)ckv.stride(0), bf(kv_ln), bf(q), (long)q.stride(0), (long)qpe_off,
                       pos.data_ptr<int>(), cos_sin.data_ptr<float>(), slots.data_ptr<int64_t>(), bf(cache), (int)T,
                       (int)H, (int)DL, (int)DR, (int)cos_sin.size(0), (long)(cache.size(0) * 64), (float)eps,
                       cur_stream());
}

// q_lat / out [H, T, DL]; q_pe rows of q (row stride ldqpe = q_pe.stride(0)) as [T, H * DR]
void mla_attn(const at::Tensor& q_lat, const at::Tensor& q_pe, const at::Tensor& cache, const at::Tensor& block_tables,
              const at::Tensor& cu_q, const at::Tensor& ctx_lens, at::Tensor& out, at::Tensor& ws_o, at::Tensor& ws_ml,
              int64_t pages_per_part, int64_t nparts, double scale, int64_t wide) {
  CHECK_BF16(q_lat);
  CHECK_BF16(q_pe);
  CHECK_BF16(cache);
  CHECK_BF16(out);
  CHECK_DT(block_tables, at::kInt);
  CHECK_DT(cu_q, at::kInt);
  CHECK_DT(ctx_lens, at::kInt);
  CHECK_DT(ws_o, at::kFloat);
  CHECK_DT(ws_ml, at::kFloat);
  XCHECK(all_contig_gpu(q_lat, cache, block_tables, cu_q, ctx_lens, out, ws_o, ws_ml), "mla_attn: contiguous GPU");
  XCHECK(q_pe.is_cuda() && q_pe.dim() == 2 && q_pe.stride(1) == 1 && q_pe.stride(0) % 8 == 0, "mla_attn: q_pe rows");
  XCHECK(q_lat.dim() == 3 && cache.dim() == 3 && cache.size(1) == 64, "mla_attn: q_lat [H, T, DL], cache [pages, 64, DL+DR]");
  const int64_t H = q_lat.size(0), T = q_lat.size(1), DL = q_lat.size(2), DR = cache.size(2) - DL;
  const int64_t B = ctx_lens.numel();
  XCHECK(q_pe.size(0) == T && q_pe.size(1) >= H * DR && out.sizes() == q_lat.sizes(), "mla_attn: shapes");
  XCHECK(cu_q.numel() == B + 1 && block_tables.dim() == 2 && block_tables.size(0) == B, "mla_attn: batch tensors");
  XCHECK(nparts == 1 || (ws_o.numel() >= T * H * nparts * DL && ws_ml.numel() >= T * H * nparts * 2),
         "mla_attn: split-KV workspace too small");
  const int rc = xot::launch_mla_attn(bf(q_lat), bf(q_pe), (long)q_pe.stride(0), bf(cache),
                                      block_tables.data_ptr<int>(), (int)block_tables.size(1), cu_q.data_ptr<int>(),
                                      ctx_lens.data_ptr<int>(), (int)B, (int)T, (int)H, (int)DL, (int)DR, bf(out),
                                      ws_o.data_ptr<float>(), ws_ml.data_ptr<float>(), (int)pages_per_part,
                                      (int)nparts, (float)scale, (int)cache.size(0), (int)wide, cur_stream());
  XCHECK(rc == 0, "mla_attn: unsupported DL=", DL, " DR=", DR);
}

void moe_combine(const at::Tensor& y, const at::Tensor& slot_of, const at::Tensor& topw, at::Tensor& h,
                 int64_t splits) {
  CHECK_GPU(y);
  CHECK_DT(y, at::kFloat);
  CHECK_BF16(h);
  XCHECK(all_contig_gpu(y, slot_of, topw, h), "moe_combine: tensors must be contiguous GPU");
  const int64_t T = h.size(0), D = h.size(1), k = slot_of.numel() / T;
  XCHECK(splits >= 1 && D % 8 == 0 && y.size(1) == D && y.size(0) == splits * T * k && topw.numel() == T * k,
         "moe_combine: shapes");
  xot::launch_moe_combine(y.data_ptr<float>(), slot_of.data_ptr<int>(), topw.data_ptr<float>(), bf(h), (int)T, (int)k,
                          (int)D, (int)splits, (long)(T * k * D), cur_stream());
}

void splitk_silu(const at::Tensor& ws, int64_t S, at::Tensor& y) {
  CHECK_DT(ws, at::kFloat);
  CHECK_BF16(y);
  XCHECK(all_contig_gpu(ws, y) && y.dim() == 2, "splitk_silu: contiguous GPU tensors, y 2-D");
  const int64_t M = y.size(0), N = 2 * y.size(1);
  XCHECK(S >= 1 && N % 32 == 0 && ws.numel() >= S * M * N, "splitk_silu: slabs must hold S x M x 2*cols");
  xot::launch_splitk_silu(ws.data_ptr<float>(), (int)S, (int)M, (int)N, bf(y), cur_stream());
}

void moe_combine_norm(const at::Tensor& y, const at::Tensor& slot_of, const at::Tensor& topw, at::Tensor& h,
                      int64_t splits, const at::Tensor& ln_w, at::Tensor& out, double eps) {
  CHECK_DT(y, at::kFloat);
  CHECK_BF16(h);
  CHECK_BF16(ln_w);
  CHECK_BF16(out);
  XCHECK(all_contig_gpu(y, slot_of, topw, h, ln_w, out), "moe_combine_norm: tensors must be contiguous GPU");
  const int64_t T = h.size(0), D = h.size(1), k = slot_of.numel() / T;
  XCHECK(splits >= 1 && D % 8 == 0 && y.size(1) == D && y.size(0) == splits * T * k && topw.numel() == T * k &&
             ln_w.numel() == D && out.sizes() == h.sizes(),
         "moe_combine_norm: shapes");
  const int rc = xot::launch_moe_combine_norm(y.data_ptr<float>(), slot_of.data_ptr<int>(), topw.data_ptr<float>(),
                                              bf(h), bf(ln_w), bf(out), (int)T, (int)k, (int)D, (int)splits,
                                              (long)(T * k * D), (float)eps, cur_stream());
  XCHECK(rc == 0, "moe_combine_norm: unsupported D=", D);
}

void attn_decode(const at::Tensor& q, const at::Tensor& k_cache, const at::Tensor& v_cache,
                 const at::Tensor& block_tables, const at::Tensor& ctx_lens, at::Tensor& out, at::Tensor& ws_o,
                 at::Tensor& ws_ml, int64_t pages_per_part, int64_t nparts, double scale, int64_t algo,
                 bool merge) {
  CHECK_BF16(q);
  CHECK_BF16(k_cache);
  CHECK_BF16(v_cache);
  CHECK_BF16(out);
  CHECK_DT(block_tables, at::kInt);
  CHECK_DT(ctx_lens, at::kInt);
  CHECK_DT(ws_o, at::kFloat);
  CHECK_DT(ws_ml, at::kFloat);
  XCHECK(all_contig_gpu(q, k_cache, v_cache, block_tables, ctx_lens, out, ws_o, ws_ml),
         "attn_decode: all tensors must be contiguous GPU tensors");
  XCHECK(q.dim() == 3 && k_cache.dim() == 4 && v_cache.dim() == 4, "attn_decode: q [B,H,Dh], caches 4-D");
  const int64_t B = q.size(0), H = q.size(1), Dh = q.size(2), Hkv = k_cache.size(1), nb = k_cache.size(0);
  XCHECK(k_cache.size(2) == 64 && k_cache.size(3) == Dh && v_cache.size(2) == Dh && v_cache.size(3) == 64 &&
             v_cache.size(0) == nb && v_cache.size(1) == Hkv,
         "attn_decode: cache layout K[nb,Hkv,64,Dh] V[nb,Hkv,Dh,64]");
  XCHECK(block_tables.dim() == 2 && block_tables.size(0) >= B && ctx_lens.numel() >= B, "attn_decode: tables");
  XCHECK(out.numel() == B * H * Dh, "attn_decode: out shape");
  XCHECK(pages_per_part >= 1 && nparts >= 1, "attn_decode: bad partitioning");
  if (nparts > 1)
    XCHECK(ws_o.numel() >= B * H * nparts * Dh && ws_ml.numel() >= B * H * nparts * 2, "attn_decode: workspace small");
  const int rc = xot::launch_attn_decode(bf(q), bf(k_cache), bf(v_cache), block_tables.data_ptr<int32_t>(),
                                         (int)block_tables.size(1), ctx_lens.data_ptr<int32_t>(), bf(out),
                                         ws_o.data_ptr<float>(), ws_ml.data_ptr<float>(), (int)B, (int)H, (int)Hkv,
                                         (int)Dh, (int)pages_per_part, (int)nparts, (float)scale, (int)nb, (int)algo,
                                         cur_stream(), merge);
  XCHECK(rc == 0, "attn_decode: unsupported H=", H, " Hkv=", Hkv, " Dh=", Dh);
}

// the partition merge attn_decode(merge = false) left out: out [B, H, Dh] from ws_o / ws_ml
void attn_decode_merge(const at::Tensor& ws_o, const at::Tensor& ws_ml, const at::Tensor& ctx_lens, at::Tensor& out,
                       int64_t pages_per_part, int64_t nparts) {
  CHECK_BF16(out);
  CHECK_DT(ws_o, at::kFloat);
  CHECK_DT(ws_ml, at::kFloat);
  CHECK_DT(ctx_lens, at::kInt);
  XCHECK(all_contig_gpu(ws_o, ws_ml, ctx_lens, out) && out.dim() == 3, "attn_decode_merge: contiguous GPU, out [B,H,Dh]");
  const int64_t B = out.size(0), H = out.size(1), Dh = out.size(2);
  XCHECK(Dh == 128 || Dh == 64, "attn_decode_merge: Dh");
  XCHECK(ws_o.numel() >= B * H * nparts * Dh && ws_ml.numel() >= B * H * nparts * 2 && ctx_lens.numel() >= B,
         "attn_decode_merge: workspace");
  xot::launch_attn_decode_merge(ws_o.data_ptr<float>(), ws_ml.data_ptr<float>(), ctx_lens.data_ptr<int32_t>(), bf(out),
                                (int)B, (int)H, (int)Dh, (int)nparts, (int)pages_per_part, cur_stream());
}

// o_proj of a batch-1 decode step on the pre-shuffled weight w [N, H*Dh], its input row merged from the attention's
// partitions (ws_o / ws_ml, row 0) in the prologue; writes `splits` fp32 slabs into ws (no reduce)
void gemm_stream_merge(const at::Tensor& w, at::Tensor& ws, int64_t ntw, int64_t splits, const at::Tensor& ws_o,
                       const at::Tensor& ws_ml, const at::Tensor& ctx_lens, int64_t pages_per_part, int64_t nparts,
                       int64_t Dh) {
  CHECK_BF16(w);
  CHECK_DT(ws, at::kFloat);
  CHECK_DT(ws_o, at::kFloat);
  CHECK_DT(ws_ml, at::kFloat);
  CHECK_DT(ctx_lens, at::kInt);
  XCHECK(all_contig_gpu(w, ws, ws_o, ws_ml, ctx_lens) && w.dim() == 2, "gemm_stream_merge: contiguous GPU tensors");
  const int64_t N = w.size(0), K = w.size(1);
  XCHECK(Dh > 0 && K % Dh == 0 && ws_o.numel() >= (K / Dh) * nparts * Dh && ws_ml.numel() >= (K / Dh) * nparts * 2,
         "gemm_stream_merge: attention workspace");
  xot::NormPro np{};
  np.mo = ws_o.data_ptr<float>();
  np.ml = ws_ml.data_ptr<float>();
  np.ctx = ctx_lens.data_ptr<int32_t>();
  np.nparts = (int)nparts;
  np.ppp = (int)pages_per_part;
  np.dh = (int)Dh;
  const int rc = xot::launch_gemm_stream_merge(bf(w), ws.data_ptr<float>(), ws.numel(), (int)N, (int)K, (int)ntw,
                                               (int)splits, np, cur_stream());
  XCHECK(rc == 0, "gemm_stream_merge: unsupported N=", N, " K=", K, " ntw=", ntw, " splits=", splits);
}

// training attention: 2-D token-major views ([B*L, n*Dh] rows, unit inner stride; row strides may differ,
// e.g. slices of the fused qkv projection)
static void check_rows(const at::Tensor& t, int64_t rows, int64_t cols, const char* what) {
  CHECK_BF16(t);
  XCHECK(t.dim() == 2 && t.size(0) == rows && t.size(1) == cols && t.stride(1) == 1 && t.stride(0) % 8 == 0,
         "attn_train: bad ", what, " view");
}

static void check_trans(const at::Tensor& t, int64_t B, int64_t n, int64_t Dh, int64_t Lp, const char* what) {
  CHECK_BF16(t);
  XCHECK(t.is_contiguous() && t.numel() == B * n * Dh * Lp, "attn_train: bad transposed ", what, " [B, n, Dh, Lp]");
}

// [B*L, n*Dh] token-major view -> [B, n, Dh, Lp] (tokens contiguous, zero past L)
void attn_train_transpose(const at::Tensor& x, at::Tensor& xt, int64_t B, int64_t L, int64_t Lp, int64_t n,
                          int64_t Dh) {
  check_rows(x, B * L, n * Dh, "x");
  check_trans(xt, B, n, Dh, Lp, "xt");
  const int rc = xot::launch_attn_train_transpose(bf(x), x.stride(0), bf(xt), (int)B, (int)L, (int)Lp, (int)n,
                                                  (int)Dh, cur_stream());
  XCHECK(rc == 0, "attn_train_transpose: unsupported Dh=", Dh, " Lp=", Lp);
}

void attn_train_fwd(const at::Tensor& q, const at::Tensor& k, const at::Tensor& vt, at::Tensor& o, at::Tensor& lse2,
                    int64_t B, int64_t L, int64_t Lp, int64_t H, int64_t Hkv, int64_t Dh, double scale,
                    bool causal) {
  check_rows(q, B * L, H * Dh, "q");
  check_rows(k, B * L, Hkv * Dh, "k");
  check_trans(vt, B, Hkv, Dh, Lp, "vt");
  check_rows(o, B * L, H * Dh, "o");
  CHECK_GPU(lse2);
  CHECK_DT(lse2, at::kFloat);
  XCHECK(lse2.is_contiguous() && lse2.numel() == B * H * L, "attn_train_fwd: lse2 [B, H, L]");
  const int rc = xot::launch_attn_train_fwd(bf(q), q.stride(0), bf(k), k.stride(0), bf(vt), (int)Lp, bf(o),
                                            o.stride(0), lse2.data_ptr<float>(), (int)B, (int)L, (int)H, (int)Hkv,
                                            (int)Dh, (float)scale, causal, cur_stream());
  XCHECK(rc == 0, "attn_train_fwd: unsupported H=", H, " Hkv=", Hkv, " Dh=", Dh);
}

void attn_train_bwd(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, const at::Tensor& o,
                    const at::Tensor& dout, const at::Tensor& lse2, at::Tensor& delta, at::Tensor& dq, at::Tensor& dk,
                    at::Tensor& dv, at::Tensor& ws, int64_t B, int64_t L, int64_t Lp, int64_t H, int64_t Hkv,
                    int64_t Dh, double scale) {
  // the kernels read the transposed operands straight from their row tiles in LDS (ds_read_b64_tr_b16)
  check_rows(q, B * L, H * Dh, "q");
  check_rows(k, B * L, Hkv * Dh, "k");
  check_rows(v, B * L, Hkv * Dh, "v");
  check_rows(o, B * L, H * Dh, "o");
  check_rows(dout, B * L, H * Dh, "dout");
  check_rows(dq, B * L, H * Dh, "dq");
  check_rows(dk, B * L, Hkv * Dh, "dk");
  check_rows(dv, B * L, Hkv * Dh, "dv");
  CHECK_DT(lse2, at::kFloat);
  CHECK_DT(delta, at::kFloat);
  XCHECK(lse2.is_contiguous() && delta.is_contiguous() && lse2.numel() == B * H * L && delta.numel() == B * H * L,
         "attn_train_bwd: lse2 / delta [B, H, L]");
  CHECK_GPU(ws);
  CHECK_DT(ws, at::kFloat);
  XCHECK(ws.is_contiguous() && ws.numel() >= 2 * H * B * L * Dh, "attn_train_bwd: ws needs 2 * H * B * L * Dh floats");
  const int rc = xot::launch_attn_train_bwd(
      bf(q), q.stride(0), bf(k), k.stride(0), bf(v), v.stride(0), bf(o), o.stride(0), bf(dout), dout.stride(0),
      (int)Lp, lse2.data_ptr<float>(), delta.data_ptr<float>(), bf(dq), dq.stride(0), bf(dk), dk.stride(0), bf(dv),
      dv.stride(0), ws.data_ptr<float>(), (long)ws.numel(), (int)B, (int)L, (int)H, (int)Hkv, (int)Dh, (float)scale,
      cur_stream());
  XCHECK(rc == 0, "attn_train_bwd: unsupported H=", H, " Hkv=", Hkv, " Dh=", Dh);
}

void attn_prefill(const at::Tensor& q, const at::Tensor& k_cache, const at::Tensor& v_cache,
                  const at::Tensor& block_tables, const at::Tensor& cu_q, const at::Tensor& ctx_lens, at::Tensor& out,
                  int64_t max_qlen, double scale, int64_t algo) {
  CHECK_BF16(q);
  CHECK_BF16(k_cache);
  CHECK_BF16(v_cache);
  CHECK_BF16(out);
  CHECK_DT(block_tables, at::kInt);
  CHECK_DT(cu_q, at::kInt);
  CHECK_DT(ctx_lens, at::kInt);
  XCHECK(all_contig_gpu(q, k_cache, v_cache, block_tables, cu_q, ctx_lens, out),
         "attn_prefill: all tensors must be contiguous GPU tensors");
  XCHECK(q.dim() == 3, "attn_prefill: q must be [T,H,Dh]");
  const int64_t H = q.size(1), Dh = q.size(2), Hkv = k_cache.size(1), nb = k_cache.size(0);
  const int64_t B = ctx_lens.numel();
  XCHECK(cu_q.numel() == B + 1 && block_tables.dim() == 2 && block_tables.size(0) >= B, "attn_prefill: tables");
  XCHECK(k_cache.size(2) == 64 && k_cache.size(3) == Dh && v_cache.size(2) == Dh && v_cache.size(3) == 64,
         "attn_prefill: cache layout");
  XCHECK(out.numel() == q.numel(), "attn_prefill: out shape");
  const int rc = xot::launch_attn_prefill(bf(q), bf(k_cache), bf(v_cache), block_tables.data_ptr<int32_t>(),
                                          (int)block_tables.size(1), cu_q.data_ptr<int32_t>(),
                                          ctx_lens.data_ptr<int32_t>(), bf(out), (int)B, (int)max_qlen, (int)H,
                                          (int)Hkv, (int)Dh, (float)scale, (int)nb, (int)algo, cur_stream());
  XCHECK(rc == 0, "attn_prefill: unsupported H=", H, " Hkv=", Hkv, " Dh=", Dh);
}

void sample(const at::Tensor& logits, const at::Tensor& temps, int64_t top_k, const at::Tensor& seed_off,
            at::Tensor& out, int64_t algo) {
  CHECK_GPU(logits);
  CHECK_DT(logits, at::kFloat);
  CHECK_DT(temps, at::kFloat);
  CHECK_DT(seed_off, at::kLong);
  CHECK_DT(out, at::kInt);
  XCHECK(logits.dim() == 2 && logits.stride(1) == 1, "sample: logits must be [B, V] with contiguous rows");
  const int64_t B = logits.size(0), V = logits.size(1);
  XCHECK(temps.numel() >= B && out.numel() >= B && seed_off.numel() >= 2, "sample: shape mismatch");
  // candidate scratch of the split path for small batches (graph-safe caching-allocator tensors)
  auto ck = at::empty({B * xot::SAMPLE_CAND_PER_ROW}, logits.options().dtype(at::kInt));
  auto ci = at::empty({B * xot::SAMPLE_CAND_PER_ROW}, logits.options().dtype(at::kInt));
  xot::launch_sample(logits.data_ptr<float>(), logits.stride(0), (int)B, (int)V, temps.data_ptr<float>(), (int)top_k,
                     seed_off.data_ptr<int64_t>(), out.data_ptr<int32_t>(),
                     reinterpret_cast<uint32_t*>(ck.data_ptr<int>()), ci.data_ptr<int>(), cur_stream(), (int)algo);
}

void topk_cand(const at::Tensor& logits, int64_t top_k, at::Tensor& vals, at::Tensor& idx) {
  CHECK_GPU(logits);
  CHECK_DT(logits, at::kFloat);
  CHECK_DT(vals, at::kFloat);
  CHECK_DT(idx, at::kInt);
  XCHECK(logits.dim() == 2 && logits.stride(1) == 1, "topk_cand: logits must be [B, V] with contiguous rows");
  const int64_t B = logits.size(0), V = logits.size(1);
  XCHECK(vals.dim() == 2 && vals.is_contiguous() && vals.size(0) == B && idx.sizes() == vals.sizes() &&
             idx.is_contiguous(), "topk_cand: vals / idx must be contiguous [B, kc]");
  const int rc = xot::launch_topk_cand(logits.data_ptr<float>(), logits.stride(0), (int)B, (int)V, (int)top_k,
                                       vals.data_ptr<float>(), idx.data_ptr<int32_t>(), (int)vals.size(1), cur_stream());
  XCHECK(rc == 0, "topk_cand: unsupported top_k=", top_k, " V=", V, " kc=", vals.size(1));
}

void ce_fwd(const at::Tensor& x, const at::Tensor& tgt, at::Tensor& loss, at::Tensor& lse) {
  CHECK_GPU(x);
  XCHECK(x.dim() == 2 && x.stride(1) == 1, "ce_fwd: x must be [T, V]");
  const bool f32 = x.scalar_type() == at::kFloat;
  XCHECK(f32 || x.scalar_type() == at::kBFloat16, "ce_fwd: x must be fp32 or bf16");
  CHECK_DT(tgt, at::kInt);
  CHECK_DT(loss, at::kFloat);
  CHECK_DT(lse, at::kFloat);
  const int64_t T = x.size(0);
  XCHECK(tgt.numel() == T && loss.numel() == T && lse.numel() == T, "ce_fwd: shape mismatch");
  xot::launch_ce_fwd(x.data_ptr(), f32, x.stride(0), (int)T, (int)x.size(1), tgt.data_ptr<int32_t>(),
                     loss.data_ptr<float>(), lse.data_ptr<float>(), cur_stream());
}

void ce_bwd(const at::Tensor& x, const at::Tensor& tgt, const at::Tensor& lse, const at::Tensor& gscale,
            at::Tensor& dx) {
  CHECK_GPU(x);
  XCHECK(x.dim() == 2 && x.stride(1) == 1 && dx.dim() == 2 && dx.stride(1) == 1, "ce_bwd: 2-D rows");
  const bool f32 = x.scalar_type() == at::kFloat;
  XCHECK(f32 || x.scalar_type() == at::kBFloat16, "ce_bwd: x must be fp32 or bf16");
  CHECK_BF16(dx);
  const int64_t T = x.size(0);
  XCHECK(dx.size(0) == T && dx.size(1) == x.size(1) && tgt.numel() == T && lse.numel() == T && gscale.numel() == T,
         "ce_bwd: shape mismatch");
  xot::launch_ce_bwd(x.data_ptr(), f32, x.stride(0), (int)T, (int)x.size(1), tgt.data_ptr<int32_t>(),
                     lse.data_ptr<float>(), gscale.data_ptr<float>(), bf(dx), dx.stride(0), cur_stream());
}

// AdamW of a 2-D weight [N, K] fused with its shuffle(W) / shuffle(W^T) operand images (N, K % 128 == 0)
void adamw_tiled(at::Tensor& p, const at::Tensor& g, at::Tensor& m, at::Tensor& v,
                 const c10::optional<at::Tensor>& p_bf16, at::Tensor& ws, at::Tensor& wts, double lr, double b1,
                 double b2, double eps, double wd, int64_t step, double gscale) {
  CHECK_DT(p, at::kFloat);
  CHECK_DT(m, at::kFloat);
  CHECK_DT(v, at::kFloat);
  CHECK_BF16(ws);
  CHECK_BF16(wts);
  const bool gf32 = g.scalar_type() == at::kFloat;
  XCHECK(gf32 || g.scalar_type() == at::kBFloat16, "adamw_tiled: grad must be fp32 or bf16");
  XCHECK(all_contig_gpu(p, g, m, v) && ws.is_contiguous() && wts.is_contiguous(), "adamw_tiled: contiguous GPU");
  XCHECK(p.dim() == 2, "adamw_tiled: 2-D weight");
  const int64_t N = p.size(0), K = p.size(1);
  XCHECK(g.numel() == N * K && m.numel() == N * K && v.numel() == N * K && ws.numel() == N * K &&
             wts.numel() == N * K, "adamw_tiled: shape mismatch");
  if (p_bf16.has_value()) {
    CHECK_BF16((*p_bf16));
    XCHECK(p_bf16->numel() == N * K && p_bf16->is_contiguous(), "adamw_tiled: p_bf16 shape");
  }
  const int rc = xot::launch_adamw_tiled(p.data_ptr<float>(), g.data_ptr(), gf32, m.data_ptr<float>(),
                                         v.data_ptr<float>(), bf_opt(p_bf16), bf(ws), bf(wts), (int)N, (int)K,
                                         (float)lr, (float)b1, (float)b2, (float)eps, (float)wd, (int)step,
                                         (float)gscale, cur_stream());
  XCHECK(rc == 0, "adamw_tiled: N and K must be multiples of 128");
}

// sum of squares of every tensor (bf16 or fp32, contiguous, one GPU) as a one-element fp32 tensor
at::Tensor multi_sumsq(const std::vector<at::Tensor>& ts) {
  XCHECK(!ts.empty(), "multi_sumsq: no tensors");
  std::vector<xot::SumsqBatch> batches;
  long maxn = 1;
  for (size_t i = 0; i < ts.size(); ++i) {
    const at::Tensor& t = ts[i];
    XCHECK(t.is_cuda() && t.is_contiguous() && t.device() == ts[0].device(), "multi_sumsq: contiguous GPU tensors");
    XCHECK(t.scalar_type() == at::kFloat || t.scalar_type() == at::kBFloat16, "multi_sumsq: fp32 or bf16");
    if (i % xot::SUMSQ_MAXT == 0) batches.push_back(xot::SumsqBatch{});
    xot::SumsqBatch& b = batches.back();
    b.p[b.count] = t.data_ptr();
    b.n[b.count] = t.numel();
    b.f32[b.count] = t.scalar_type() == at::kFloat;
    ++b.count;
    maxn = std::max<long>(maxn, t.numel());
  }
  const int maxc = (int)((maxn + xot::multi_sumsq_chunk() - 1) / xot::multi_sumsq_chunk());
  auto part = at::empty({xot::multi_sumsq_scratch((int)batches.size(), maxc)}, ts[0].options().dtype(at::kFloat));
  auto out = at::empty({1}, ts[0].options().dtype(at::kFloat));
  part.zero_();  // rows of a batch's unused tensor slots
  xot::launch_multi_sumsq(batches.data(), (int)batches.size(), maxc, part.data_ptr<float>(), out.data_ptr<float>(),
                          cur_stream());
  return out;
}

void adamw(at::Tensor& p, const at::Tensor& g, at::Tensor& m, at::Tensor& v, const c10::optional<at::Tensor>& p_bf16,
           double lr, double b1, double b2, double eps, double wd, int64_t step, double gscale) {
  CHECK_DT(p, at::kFloat);
  CHECK_DT(m, at::kFloat);
  CHECK_DT(v, at::kFloat);
  const bool gf32 = g.scalar_type() == at::kFloat;
  XCHECK(gf32 || g.scalar_type() == at::kBFloat16, "adamw: grad must be fp32 or bf16");
  XCHECK(all_contig_gpu(p, g, m, v), "adamw: contiguous GPU tensors");
  const int64_t n = p.numel();
  XCHECK(g.numel() == n && m.numel() == n && v.numel() == n, "adamw: shape mismatch");
  if (p_bf16.has_value()) {
    CHECK_BF16((*p_bf16));
    XCHECK(p_bf16->numel() == n && p_bf16->is_contiguous(), "adamw: p_bf16 shape");
  }
  xot::launch_adamw(p.data_ptr<float>(), g.data_ptr(), gf32, m.data_ptr<float>(), v.data_ptr<float>(),
                    bf_opt(p_bf16), n, (float)lr, (float)b1, (float)b2, (float)eps, (float)wd, (int)step,
                    (float)gscale, cur_stream());
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "xot MI355X (gfx950) kernel library";
  m.def("rmsnorm", &rmsnorm);
  m.def("rmsnorm_bwd", &rmsnorm_bwd, py::arg("x"), py::arg("w"), py::arg("dy"), py::arg("dx"), py::arg("dw"),
        py::arg("eps"), py::arg("res") = py::none());
  m.def("embedding", &embedding);
  m.def("silu_mul", &silu_mul);
  m.def("silu_mul_bwd", &silu_mul_bwd);
  m.def("rope_kv_write", &rope_kv_write);
  m.def("rope_apply", &rope_apply);
  m.def("gemm", &gemm);
  m.def("gemm_stream", &gemm_stream, py::arg("x"), py::arg("w"), py::arg("y"), py::arg("bias"), py::arg("res"),
        py::arg("ws"), py::arg("epi"), py::arg("ntw"), py::arg("splits"), py::arg("wshuf"),
        py::arg("reduce") = true);
  m.def("gemm_stream_norm", &gemm_stream_norm, py::arg("w"), py::arg("y"), py::arg("bias"), py::arg("ws"),
        py::arg("epi"), py::arg("ntw"), py::arg("splits"), py::arg("reduce"), py::arg("h"), py::arg("ws_in"),
        py::arg("s_in"), py::arg("bias_in"), py::arg("lnw"), py::arg("hout"), py::arg("eps"));
  m.def("gemm_stream8", &gemm_stream8, py::arg("x"), py::arg("w8"), py::arg("wscale"), py::arg("y"), py::arg("bias"),
        py::arg("res"), py::arg("ws"), py::arg("epi"), py::arg("ntw"), py::arg("splits"), py::arg("reduce") = true);
  m.def("relayout", &relayout, py::arg("src"), py::arg("dst"), py::arg("mode"));
  m.def("gemm_kgroup", &gemm_kgroup);
  m.def("gemm_tn", &gemm_tn, py::arg("dy"), py::arg("x"), py::arg("y"), py::arg("resid"));
  m.def("gemm_batched", &gemm_batched, py::arg("x"), py::arg("xbat"), py::arg("K"), py::arg("w"), py::arg("y"),
        py::arg("ybat"), py::arg("ldy"), py::arg("M"));
  m.def("gemm_big", &gemm_big, py::arg("x"), py::arg("w"), py::arg("y"), py::arg("bias"), py::arg("res"),
        py::arg("ws"), py::arg("epi"), py::arg("bn"), py::arg("splits"), py::arg("reduce") = true);
  m.def("splitk_resid_rmsnorm", &splitk_resid_rmsnorm);
  m.def("gemm_moe", &gemm_moe, py::arg("x"), py::arg("w"), py::arg("y"), py::arg("off"), py::arg("gather"),
        py::arg("epi"), py::arg("max_rows"), py::arg("wshuf"), py::arg("splits") = 1, py::arg("big_bm") = 0);
  m.def("moe_route", &moe_route);
  m.def("moe_route_ds", &moe_route_ds);
  m.def("mla_prep", &mla_prep);
  m.def("mla_attn", &mla_attn, py::arg("q_lat"), py::arg("q_pe"), py::arg("cache"), py::arg("block_tables"),
        py::arg("cu_q"), py::arg("ctx_lens"), py::arg("out"), py::arg("ws_o"), py::arg("ws_ml"), py::arg("pages_per_part"),
        py::arg("nparts"), py::arg("scale"), py::arg("wide") = 0);
  m.def("moe_combine", &moe_combine, py::arg("y"), py::arg("slot_of"), py::arg("topw"), py::arg("h"),
        py::arg("splits") = 1);
  m.def("attn_decode", &attn_decode, py::arg("q"), py::arg("k_cache"), py::arg("v_cache"), py::arg("block_tables"),
        py::arg("ctx_lens"), py::arg("out"), py::arg("ws_o"), py::arg("ws_ml"), py::arg("pages_per_part"),
        py::arg("nparts"), py::arg("scale"), py::arg("algo") = 2, py::arg("merge") = true);
  m.def("attn_decode_merge", &attn_decode_merge, py::arg("ws_o"), py::arg("ws_ml"), py::arg("ctx_lens"), py::arg("out"),
        py::arg("pages_per_part"), py::arg("nparts"));
  m.def("gemm_stream_merge", &gemm_stream_merge, py::arg("w"), py::arg("ws"), py::arg("ntw"), py::arg("splits"),
        py::arg("ws_o"), py::arg("ws_ml"), py::arg("ctx_lens"), py::arg("pages_per_part"), py::arg("nparts"),
        py::arg("Dh"));
  m.def("attn_prefill", &attn_prefill, py::arg("q"), py::arg("k_cache"), py::arg("v_cache"), py::arg("block_tables"),
        py::arg("cu_q"), py::arg("ctx_lens"), py::arg("out"), py::arg("max_qlen"), py::arg("scale"), py::arg("algo") = 2);
  m.def("router_logits", &router_logits);
  m.def("moe_combine_norm", &moe_combine_norm);
  m.def("splitk_silu", &splitk_silu);
  m.def("splitk_rope_kv_write", &splitk_rope_kv_write);
  m.def("attn_train_transpose", &attn_train_transpose);
  m.def("attn_train_fwd", &attn_train_fwd);
  m.def("attn_train_bwd", &attn_train_bwd);
  m.def("topk_cand", &topk_cand);
  m.def("sample", &sample, py::arg("logits"), py::arg("temps"), py::arg("top_k"), py::arg("seed_off"), py::arg("out"),
        py::arg("algo") = -1);
  m.def("ce_fwd", &ce_fwd);
  m.def("ce_bwd", &ce_bwd);
  m.def("adamw", &adamw);
  m.def("multi_sumsq", &multi_sumsq);
  m.def("adamw_tiled", &adamw_tiled);
}

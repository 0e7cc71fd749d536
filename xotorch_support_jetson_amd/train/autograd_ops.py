"""Autograd functions over the gfx950 kernel library (fp32 torch math on CPU tensors).

  RMSNormFn    forward rmsnorm kernel, backward rmsnorm_bwd kernel (dx + fp32 dw reduction)
  SiluMulFn    [gate | up] -> silu(gate) * up, backward silu_mul_bwd kernel
  RopeFn       rotate-half RoPE; backward = the inverse rotation (same kernel, sin negated)
  CrossEntropyFn  per-row loss with ignore (-100) and per-row weights; forward ce_fwd, backward ce_bwd
  AttentionFn  causal GQA self-attention: attn_train_fwd (flash-style, saves O and the row log2-sum-exp),
               backward attn_train_bwd (dQ pass with delta = rowsum(dO*O), then the dK/dV pass)
OwnLinearFn  projections on the MFMA GEMMs (shuffled operands from csrc/layout.hip); LinearFn (torch.matmul)
             only for shapes the tiles do not cover.
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from ..ops import reference as ref
from ..ops._ext import require


def _gpu(t: torch.Tensor) -> bool:
  return t.is_cuda


def _norm_dw(w, acc, dev):
  """The fp32 dw the RMSNorm backward kernel adds into: the norm weight's GradAcc buffer (zeroed on the step's
  first micro-batch; the kernel's reduce accumulates with atomics), or a fresh zeroed vector."""
  if acc is None:
    return torch.zeros(w.numel(), dtype=torch.float32, device=dev)
  if acc.fresh:
    acc.buf.zero_()
    acc.fresh = False
  return acc.buf


def _norm_dw_out(w, dw, acc):
  """The weight gradient autograd sees: none when it went into the GradAcc (then its callback fires)."""
  if acc is None:
    return dw.to(w.dtype)
  if acc.cb is not None:
    acc.cb()
  return None


class RMSNormFn(torch.autograd.Function):
  @staticmethod
  def forward(ctx, x, w, eps, acc=None):
    ctx.eps, ctx.acc = eps, acc
    ctx.save_for_backward(x, w)
    if _gpu(x):
      out = torch.empty_like(x)
      require().rmsnorm(x.contiguous(), w, out, None, None, float(eps))
      return out
    return ref.rmsnorm(x, w, eps)[0]

  @staticmethod
  def backward(ctx, dy):
    x, w = ctx.saved_tensors
    if _gpu(x):
      dx = torch.empty_like(x)
      dw = _norm_dw(w, ctx.acc, x.device)
      require().rmsnorm_bwd(x.contiguous(), w, dy.contiguous().to(x.dtype), dx, dw, float(ctx.eps))
      return dx, _norm_dw_out(w, dw, ctx.acc), None, None
    with torch.enable_grad():
      xr = x.detach().float().requires_grad_()
      wr = w.detach().float().requires_grad_()
      y = xr * torch.rsqrt(xr.pow(2).mean(-1, keepdim=True) + ctx.eps) * wr
      y.backward(dy.float())
    return xr.grad.to(x.dtype), wr.grad.to(w.dtype), None, None


class ResNormFn(torch.autograd.Function):
  """(h, rmsnorm(h)) for a residual stream h that is both normalised into a branch and carried on: the backward
  joins the two gradients in the RMSNorm backward kernel (dh = dh_carried + rmsnorm'(dxn), csrc/norm_rope.hip
  `res`) instead of autograd's separate add kernel per residual join (2 per layer and micro-batch)."""

  @staticmethod
  def forward(ctx, h, w, eps, acc=None):
    ctx.eps, ctx.acc = eps, acc
    ctx.save_for_backward(h, w)
    if _gpu(h):
      xn = torch.empty_like(h)
      require().rmsnorm(h.contiguous(), w, xn, None, None, float(eps))
    else:
      xn = ref.rmsnorm(h, w, eps)[0]
    return h.view_as(h), xn

  @staticmethod
  def backward(ctx, dh, dxn):
    h, w = ctx.saved_tensors
    if dxn is None:
      return dh, None, None, None
    if _gpu(h):
      dx = torch.empty_like(h)
      dw = _norm_dw(w, ctx.acc, h.device)
      res = dh.contiguous().to(h.dtype) if dh is not None else None
      require().rmsnorm_bwd(h.contiguous(), w, dxn.contiguous().to(h.dtype), dx, dw, float(ctx.eps), res)
      return dx, _norm_dw_out(w, dw, ctx.acc), None, None
    dx, dw, _, _ = RMSNormFn.backward(ctx, dxn)
    return (dx if dh is None else dx + dh), dw, None, None


class SiluMulFn(torch.autograd.Function):
  @staticmethod
  def forward(ctx, gu):
    ctx.save_for_backward(gu)
    if _gpu(gu):
      Fd = gu.shape[-1] // 2
      out = torch.empty(*gu.shape[:-1], Fd, dtype=gu.dtype, device=gu.device)
      require().silu_mul(gu.contiguous(), out, False)
      return out
    return ref.silu_mul(gu)

  @staticmethod
  def backward(ctx, dout):
    (gu,) = ctx.saved_tensors
    if _gpu(gu):
      dgu = torch.empty_like(gu)
      require().silu_mul_bwd(gu.contiguous(), dout.contiguous().to(gu.dtype), dgu)
      return dgu
    Fd = gu.shape[-1] // 2
    g, u = gu[..., :Fd].float(), gu[..., Fd:].float()
    sg = torch.sigmoid(g)
    d = dout.float()
    dg = d * u * (sg * (1 + g * (1 - sg)))
    du = d * g * sg
    return torch.cat([dg, du], -1).to(gu.dtype)


class RopeFn(torch.autograd.Function):
  """x [T, nh*Dh] rows; positions [T] int32."""

  @staticmethod
  def forward(ctx, x, pos, cos_sin, nh, Dh):
    ctx.save_for_backward(pos, cos_sin)
    ctx.nh, ctx.Dh = nh, Dh
    return _rope(x, pos, cos_sin, nh, Dh, False)

  @staticmethod
  def backward(ctx, dy):
    pos, cos_sin = ctx.saved_tensors
    return _rope(dy.contiguous(), pos, cos_sin, ctx.nh, ctx.Dh, True), None, None, None, None


def _rope(x, pos, cos_sin, nh, Dh, inverse):
  if _gpu(x):
    out = torch.empty(x.shape[0], nh * Dh, dtype=x.dtype, device=x.device)
    require().rope_apply(x.contiguous(), out, pos, cos_sin, int(nh), int(Dh), bool(inverse))
    return out
  return ref.rope(x.reshape(-1, nh, Dh), pos, cos_sin, inverse).reshape(x.shape[0], nh * Dh)


class CrossEntropyFn(torch.autograd.Function):
  """logits [T, V] (bf16/fp32), targets [T] int32 (<0 ignored), weights [T] fp32 -> sum_t w_t * loss_t."""

  @staticmethod
  def forward(ctx, logits, targets, weights):
    if _gpu(logits):
      T = logits.shape[0]
      loss = torch.empty(T, dtype=torch.float32, device=logits.device)
      lse = torch.empty_like(loss)
      require().ce_fwd(logits.contiguous(), targets, loss, lse)
    else:
      loss, lse = ref.cross_entropy(logits, targets)
    ctx.save_for_backward(logits, targets, lse, weights)
    return (loss * weights).sum()

  @staticmethod
  def backward(ctx, g):
    logits, targets, lse, weights = ctx.saved_tensors
    gs = (weights * g).float().contiguous()
    if _gpu(logits):
      dx = torch.empty(logits.shape, dtype=torch.bfloat16, device=logits.device)
      require().ce_bwd(logits.contiguous(), targets, lse, gs, dx)
      return dx.to(logits.dtype), None, None
    p = torch.softmax(logits.float(), -1)
    valid = targets >= 0
    oh = F.one_hot(targets.clamp(min=0).long(), logits.shape[-1]).float()
    d = (p - oh) * gs[:, None] * valid[:, None].float()
    return d.to(logits.dtype), None, None


class AttentionFn(torch.autograd.Function):
  """q [B*L, H*Dh], k / v [B*L, Hkv*Dh] (token-major, may be strided row views) -> o [B*L, H*Dh]."""

  @staticmethod
  def forward(ctx, q, k, v, B, L, H, Hkv, Dh, scale=None):
    scale = Dh ** -0.5 if scale is None else float(scale)
    Lp = -(-L // 64) * 64
    ctx.dims = (B, L, Lp, H, Hkv, Dh, scale)
    if _gpu(q):
      C = require()
      o = torch.empty(B * L, H * Dh, dtype=q.dtype, device=q.device)
      lse2 = torch.empty(B * H * L, dtype=torch.float32, device=q.device)
      vt = _transposed(C, v, B, L, Lp, Hkv, Dh)
      C.attn_train_fwd(q, k, vt, o, lse2, B, L, Lp, H, Hkv, Dh, scale, True)
      ctx.save_for_backward(q, k, v, o, lse2)
      return o
    ctx.save_for_backward(q, k, v)
    return _attn_ref(q, k, v, B, L, H, Hkv, Dh, scale)

  @staticmethod
  def backward(ctx, do):
    B, L, Lp, H, Hkv, Dh, scale = ctx.dims
    if _gpu(do):
      C = require()
      q, k, v, o, lse2 = ctx.saved_tensors
      do = do.contiguous().to(q.dtype)
      dq = torch.empty(B * L, H * Dh, dtype=q.dtype, device=q.device)
      dk = torch.empty(B * L, Hkv * Dh, dtype=q.dtype, device=q.device)
      dv = torch.empty_like(dk)
      delta = torch.empty_like(lse2)
      ws = torch.empty(2 * H * B * L * Dh, dtype=torch.float32, device=q.device)  # per-query-head dK/dV partials
      C.attn_train_bwd(q, k, v, o, do, lse2, delta, dq, dk, dv, ws, B, L, Lp, H, Hkv, Dh, scale)
      return dq, dk, dv, None, None, None, None, None, None
    q, k, v = ctx.saved_tensors
    with torch.enable_grad():
      qr, kr, vr = (t.detach().float().requires_grad_() for t in (q, k, v))
      y = _attn_ref(qr, kr, vr, B, L, H, Hkv, Dh, scale)
      y.backward(do.float())
    return qr.grad.to(q.dtype), kr.grad.to(k.dtype), vr.grad.to(v.dtype), None, None, None, None, None, None


def _transposed(C, x, B, L, Lp, n, Dh):
  """[B*L, n*Dh] token-major -> [B, n, Dh, Lp] (the operand MFMA reads by column), zero past L."""
  xt = torch.empty(B, n, Dh, Lp, dtype=x.dtype, device=x.device)
  C.attn_train_transpose(x, xt, B, L, Lp, n, Dh)
  return xt


def _attn_ref(q, k, v, B, L, H, Hkv, Dh, scale=None):
  """fp32 causal GQA attention (reference / CPU path)."""
  qh = q.float().reshape(B, L, H, Dh).transpose(1, 2)
  kh = k.float().reshape(B, L, Hkv, Dh).transpose(1, 2).repeat_interleave(H // Hkv, dim=1)
  vh = v.float().reshape(B, L, Hkv, Dh).transpose(1, 2).repeat_interleave(H // Hkv, dim=1)
  a = F.scaled_dot_product_attention(qh, kh, vh, is_causal=True, scale=scale)
  return a.transpose(1, 2).reshape(B * L, H * Dh).to(q.dtype)


def attention(q, k, v, B, L, H, Hkv, Dh, scale=None):
  return AttentionFn.apply(q, k, v, B, L, H, Hkv, Dh, scale)


ATTN_DH = (64, 128, 192)  # head sizes of the MFMA training attention kernels


def attention_qk_v(q, k, v, B, L, H, dqk, dv, scale):
  """Causal attention with q / k heads of dqk and v heads of dv <= dqk (DeepSeek MLA in its expanded form:
  192 / 128): v is zero-padded per head to dqk so one kernel head size serves both products, and the output's
  padding columns are dropped (their gradient never reaches v).  q, k [T, H*dqk], v [T, H*dv] -> [T, H*dv]."""
  T = q.shape[0]
  vp = F.pad(v.reshape(T, H, dv), (0, dqk - dv)).reshape(T, H * dqk) if dv < dqk else v
  o = attention(q.contiguous(), k.contiguous(), vp.contiguous(), B, L, H, H, dqk, scale)
  return o.view(T, H, dqk)[..., :dv].reshape(T, H * dv)


def rmsnorm(x, w, eps, acc=None):
  """acc: the weight's fp32 GradAcc (GPU: dw accumulates there across micro-batches, no autograd gradient)."""
  return RMSNormFn.apply(x, w, eps, acc)


def res_rmsnorm(h, w, eps, acc=None):
  """(h, rmsnorm(h, w)): use the returned h downstream so the residual gradient joins in the norm's backward."""
  return ResNormFn.apply(h, w, eps, acc)


def silu_mul(gu):
  return SiluMulFn.apply(gu)


def rope(x, pos, cos_sin, nh, Dh):
  return RopeFn.apply(x, pos, cos_sin, nh, Dh)


def cross_entropy(logits, targets, weights):
  return CrossEntropyFn.apply(logits, targets, weights)


class GradAcc:
  """Gradient buffer of one projection weight with fused accumulation (see LinearFn).  `fresh`: no
  micro-batch has written it since the last zero_grad (the next one writes with beta = 0, so the
  buffer never needs zeroing); `cb`: called after each accumulation (data parallelism hooks here)."""

  def __init__(self, name: str, w: torch.Tensor):
    self.name = name
    self.buf = torch.empty_like(w, dtype=torch.bfloat16)
    self.fresh = True
    self.cb = None


class EmbedAccFn(torch.autograd.Function):
  """h = W[ids] (an untied input embedding) whose backward adds the dh rows into its GradAcc buffer (fp32 [V, D],
  index_add_) instead of autograd's per-micro-batch dense [V, D] gradient (a zero fill of the whole table, a
  sort-and-scatter, then an add of the table into .grad for every micro-batch after the first)."""

  @staticmethod
  def forward(ctx, ids, w, acc):
    ctx.save_for_backward(ids)
    ctx.acc = acc
    return F.embedding(ids, w)

  @staticmethod
  def backward(ctx, dh):
    (ids,) = ctx.saved_tensors
    acc = ctx.acc
    if acc.fresh:
      acc.buf.zero_()
      acc.fresh = False
    acc.buf.index_add_(0, ids.reshape(-1), dh.reshape(-1, dh.shape[-1]).float())
    if acc.cb is not None:
      acc.cb()
    return None, None, None


def embed_acc(ids, w, acc):
  return EmbedAccFn.apply(ids, w, acc)


class StackAccFn(torch.autograd.Function):
  """Per-expert views of an expert stack [E, R, C] whose backward adds each routed expert's gradient
  straight into the stack's GradAcc buffer (zeroed once per step) and returns no gradient for the stack:
  plain unbind would stack a full [E, R, C] gradient (zeros for idle experts) per micro-batch and
  then add it into .grad."""

  @staticmethod
  def forward(ctx, w, acc):
    ctx.acc = acc
    ctx.set_materialize_grads(False)
    return tuple(w[e] for e in range(w.shape[0]))

  @staticmethod
  def backward(ctx, *gs):
    acc = ctx.acc
    if acc.fresh:
      acc.buf.zero_()
      acc.fresh = False
    for e, g in enumerate(gs):
      if g is not None:
        acc.buf[e].add_(g)
    if acc.cb is not None:
      acc.cb()
    return None, None


def unbind_acc(w, acc):
  return StackAccFn.apply(w, acc)


class LinearFn(torch.autograd.Function):
  """y = x @ W^T (+ h).  The backward accumulates dW = dy^T x straight into the weight's GradAcc buffer
  (the GEMM's beta = 1 after the first micro-batch) and returns no gradient for W, instead of
  materialising dW and adding it into .grad -- the add alone moved 3 x 16 GB per micro-batch for
  Llama-3-8B (6 % of the train step in the kernel profile)."""

  @staticmethod
  def forward(ctx, x, w, h, acc):
    ctx.save_for_backward(x, w)
    ctx.acc = acc
    ctx.has_h = h is not None
    return torch.addmm(h, x, w.t()) if h is not None else x @ w.t()

  @staticmethod
  def backward(ctx, dy):
    x, w = ctx.saved_tensors
    acc = ctx.acc
    dy = dy.contiguous()
    dx = dy @ w
    if acc.fresh:
      torch.mm(dy.t(), x, out=acc.buf)
      acc.fresh = False
    else:
      acc.buf.addmm_(dy.t(), x)
    if acc.cb is not None:
      acc.cb()
    return dx, None, (dy if ctx.has_h else None), None


def linear_acc(x, w, acc, h=None):
  return LinearFn.apply(x, w, h, acc)


# ------------------------------------------------------------------ projections on the kernel library
def relayout(src: torch.Tensor, mode: int, out: torch.Tensor | None = None) -> torch.Tensor:
  """csrc/layout.hip: 0 shuffle(src), 1 shuffle(src^T), 2 src^T (row-major); src [R, C] bf16 with unit column
  stride.  The shuffled results are tagged with the "stream" layout the GEMM dispatch (ops/linear.py) reads."""
  R, C = src.shape
  if out is None:
    out = torch.empty((R, C) if mode == 0 else (C, R), dtype=torch.bfloat16, device=src.device)
  require().relayout(src, out, mode)
  if mode != 2:
    out.xot_layout = "stream"
  return out


class TrainWeight:
  """A projection weight W [N, K] in the two operand layouts of the own GEMMs, refreshed after every optimizer
  step (`refresh`, ~2 x 2 bytes x |W| of HBM traffic): ws = shuffle(W) for y = x W^T and wts = shuffle(W^T)
  for dX = dY W.  `ok` is False for shapes the tiles do not cover (then the projection stays on torch)."""

  def __init__(self, w: torch.Tensor):
    self.w = w
    N, K = w.shape
    self.ok = w.is_cuda and w.dim() == 2 and N % 128 == 0 and K % 128 == 0
    if self.ok:
      self.ws = torch.empty_like(w, dtype=torch.bfloat16, requires_grad=False)
      self.wts = torch.empty(K, N, dtype=torch.bfloat16, device=w.device)
      self.refresh()

  @torch.no_grad()
  def refresh(self) -> None:
    if self.ok:
      relayout(self.w.detach(), 0, self.ws)
      relayout(self.w.detach(), 1, self.wts)


def pad_rows(t: torch.Tensor, mult: int = 128, value=0) -> torch.Tensor:
  """t with its rows (dim 0) padded to a multiple of `mult` (`value` rows), or t itself when aligned.  Zero rows
  are exact for the weight-gradient GEMMs: a zero dY (or dlogits) row adds nothing to dW = dY^T X."""
  T = t.shape[0]
  Tp = -(-T // mult) * mult
  if Tp == T:
    return t
  out = torch.full((Tp,) + tuple(t.shape[1:]), value, dtype=t.dtype, device=t.device) if value else \
      torch.zeros((Tp,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
  out[:T] = t
  return out


# Weight gradients on a side stream (XOT_DW_STREAM=0: inline).  dW is off the backward's critical path (only the
# optimizer step reads it), so the dW GEMMs and their relayouts run beside the dX chain: the tail rounds of one
# GEMM (qkv dW: 384 tiles = 1.5 rounds of 256 CUs; down dX / dW: 3.5 rounds) and the chain's memory-bound kernels
# (SiLU / RMSNorm / attention backward, relayouts) fill each other's idle CUs.  Every reader of a GradAcc buffer
# on the main stream joins first (join_dw_stream: trainer.grads, the optimizer step, the data-parallel buckets).
DW_STREAM = os.environ.get("XOT_DW_STREAM", "1") != "0"
_DW_STREAMS: dict = {}


def _dw_stream(dev: torch.device):
  s = _DW_STREAMS.get(dev.index)
  if s is None:
    s = _DW_STREAMS[dev.index] = torch.cuda.Stream(device=dev)
  return s


def join_dw_stream() -> None:
  """The current stream waits for every weight gradient queued on the side streams so far."""
  for s in _DW_STREAMS.values():
    torch.cuda.current_stream(s.device).wait_stream(s)


def own_dw(dy: torch.Tensor, x: torch.Tensor, acc: "GradAcc", cb: bool = True) -> None:
  """acc.buf (+)= dY^T X on the own tiles (on the side stream when DW_STREAM), then acc.cb (if `cb`)."""
  if not (DW_STREAM and dy.is_cuda):
    _dw(dy, x, acc)
    if cb and acc.cb is not None:
      acc.cb()
    return
  side = _dw_stream(dy.device)
  side.wait_stream(torch.cuda.current_stream(dy.device))  # dy and x are ready
  with torch.cuda.stream(side):
    _dw(dy, x, acc)
  dy.record_stream(side)  # allocated on the main stream, read by the side stream: no reuse before it ran
  x.record_stream(side)
  if cb and acc.cb is not None:
    acc.cb()  # on the main stream: a callback that reads acc.buf joins the side stream first


# Weight gradients straight from the token-major dY and X (csrc/gemm_w4.hip TN: both operands staged as [64 tokens]
# row tiles by LDS-DMA, MFMA fragments read transposed out of LDS with ds_read_b64_tr_b16): no dY^T / shuffle(X^T)
# images in HBM (~1.1 GB of relayout traffic per layer and 4096-token micro-batch on Llama-3-8B, and their transient
# buffers).  The TN tile runs 5-10 % slower than the pre-shuffled one and the relayouts cost about that much: the step
# is the same (706-708 vs 709 ms, profiles/r6/train/tn/).  XOT_DW_TN=0: relayouts + the pre-shuffled tile.
DW_TN = os.environ.get("XOT_DW_TN", "1") != "0"


def dw_tn(dy: torch.Tensor, x: torch.Tensor, out: torch.Tensor, accumulate: bool) -> bool:
  """out (+)= dY^T X on the TN tile when the shapes allow it (dY [T, M], X [T, N], M and N multiples of 256; T is
  zero-padded to 64).  False: not taken (the caller builds the relayout images)."""
  if not (DW_TN and dy.is_cuda and dy.shape[1] % 256 == 0 and x.shape[1] % 256 == 0):
    return False
  dy, x = pad_rows(dy, 64), pad_rows(x, 64)
  if dy.stride(1) != 1 or dy.stride(0) % 8:
    dy = dy.contiguous()
  if x.stride(1) != 1 or x.stride(0) % 8:
    x = x.contiguous()
  if dy.shape[0] * max(dy.stride(0), x.stride(0)) * 2 >= (1 << 31):  # the tile's 32-bit LDS-DMA byte offsets
    return False
  require().gemm_tn(dy, x, out, accumulate)
  return True


def _dw(dy: torch.Tensor, x: torch.Tensor, acc: "GradAcc") -> None:
  if dw_tn(dy, x, acc.buf, not acc.fresh):
    acc.fresh = False
  else:
    _dw_gemm(*_dw_operands(dy, x), acc)


def _dw_operands(dy: torch.Tensor, x: torch.Tensor):
  """dY^T [N, T] row-major and shuffle(X^T) [K, T] for the dW GEMM; they need T % 128, so ragged token counts (the
  reference's batch-size-1 JSONL lengths) are zero-padded to 128 rows first."""
  dy, x = pad_rows(dy), pad_rows(x)
  return relayout(dy, 2), relayout(x, 1)


def _dw_gemm(dyt: torch.Tensor, xts: torch.Tensor, acc: "GradAcc") -> None:
  """acc.buf (+)= dyt . xts^T on the own tiles (plain store on the step's first micro-batch, then accumulate)."""
  from ..ops.linear import linear
  if acc.fresh:
    linear(dyt, xts, out=acc.buf)
    acc.fresh = False
  else:
    linear(dyt, xts, residual=acc.buf, epi="resid", out=acc.buf)


class OwnLinearFn(torch.autograd.Function):
  """LinearFn on the kernel library's MFMA GEMMs (gemm_big / stream-K / weight-streaming, chosen per shape by
  ops/linear.py's policy) instead of hipBLASLt:
    forward   y  = x . shuffle(W)^T (+ h: the residual epilogue)
    backward  dX = dY . shuffle(W^T)^T
              dW = dY^T . shuffle(X^T)^T into the GradAcc buffer (plain store on the first micro-batch of a
                   step, residual epilogue acc += ... after), with dY^T and shuffle(X^T) built per micro-batch
                   by csrc/layout.hip (about 2 x T x (N + K) x 2 bytes each) -- or, by default, straight from dY
                   and X on the four-wave TN tile (dw_tn) -- on the weight-gradient side stream (DW_STREAM above)."""

  @staticmethod
  def forward(ctx, x, w, tw, h, acc):
    from ..ops.linear import linear
    x = x if (x.stride(1) == 1 and x.stride(0) % 8 == 0) else x.contiguous()
    ctx.save_for_backward(x)
    ctx.tw, ctx.acc, ctx.has_h = tw, acc, h is not None
    if h is not None:
      return linear(x, tw.ws, residual=h.contiguous(), epi="resid")
    return linear(x, tw.ws)

  @staticmethod
  def backward(ctx, dy):
    from ..ops.linear import linear
    (x,) = ctx.saved_tensors
    tw, acc = ctx.tw, ctx.acc
    dy = dy.contiguous()
    dx = linear(dy, tw.wts)
    own_dw(dy, x, acc)
    return dx, None, None, (dy if ctx.has_h else None), None


def linear_own(x, w, tw, acc, h=None):
  return OwnLinearFn.apply(x, w, tw, h, acc)


class SiluDownFn(torch.autograd.Function):
  """y = (silu(gate) * up) . W_down^T (+ h): SiluMulFn and the down projection's OwnLinearFn in one autograd node
  (the backward: dA = dY . W_down on the own tiles, then silu_mul_bwd at ~6 TB/s).  (The SiLU backward in the dA
  GEMM's epilogue was measured slower -- 728-730 vs 721 ms per Llama-3-8B step, profiles/r5/train/silu_bwd_fused/:
  the gate / up reads and two outputs sat at the tail of every tile on the dX chain's critical path -- and removed.)"""

  @staticmethod
  def forward(ctx, gu, w, tw, h, acc):
    from ..ops.linear import linear
    gu = gu.contiguous()
    F = gu.shape[1] // 2
    a = torch.empty(gu.shape[0], F, dtype=gu.dtype, device=gu.device)
    require().silu_mul(gu, a, False)
    ctx.save_for_backward(gu, a)
    ctx.tw, ctx.acc, ctx.has_h = tw, acc, h is not None
    if h is not None:
      return linear(a, tw.ws, residual=h.contiguous(), epi="resid")
    return linear(a, tw.ws)

  @staticmethod
  def backward(ctx, dy):
    from ..ops.linear import linear
    gu, a = ctx.saved_tensors
    tw, acc = ctx.tw, ctx.acc
    dy = dy.contiguous()
    dgu = torch.empty_like(gu)
    require().silu_mul_bwd(gu, linear(dy, tw.wts), dgu)
    own_dw(dy, a, acc)
    return dgu, None, None, (dy if ctx.has_h else None), None


def silu_down_own(gu, w, tw, acc, h=None):
  return SiluDownFn.apply(gu, w, tw, h, acc)


class StackWeight:
  """An expert stack W [E, N, K] in the grouped GEMMs' operand layouts (per expert, refreshed after every
  optimizer step): ws[e] = shuffle(W[e]) (forward), wts[e] = shuffle(W[e]^T) (input gradient)."""

  def __init__(self, w: torch.Tensor):
    self.w = w
    E, N, K = w.shape
    self.ok = w.is_cuda and N % 128 == 0 and K % 128 == 0
    if self.ok:
      self.ws = torch.empty(E, N, K, dtype=torch.bfloat16, device=w.device)
      self.wts = torch.empty(E, K, N, dtype=torch.bfloat16, device=w.device)
      self.ws.xot_layout = self.wts.xot_layout = "stream"
      self.refresh()

  @torch.no_grad()
  def refresh(self) -> None:
    if self.ok:
      w = self.w.detach()
      for e in range(w.shape[0]):
        relayout(w[e], 0, self.ws[e])
        relayout(w[e], 1, self.wts[e])


def _grouped(x, w, off, max_rows):
  """y[rows of expert e] = x[rows] . w[e]^T over the padded slot layout (csrc: gemm_moe; gemm_big tiles when
  the output width allows, else the weight-streaming kernel)."""
  E, N, K = w.shape
  y = torch.empty(x.shape[0], N, dtype=torch.bfloat16, device=x.device)
  bm = 256 if N % 256 == 0 else 0
  require().gemm_moe(x, w, y, off, None, 0, max_rows, True, 1, bm)
  return y


class GroupedExpertsFn(torch.autograd.Function):
  """The routed experts of one MoE layer over a padded slot layout, all on the kernel library and without
  a host sync: xs [P, D] holds every (token, choice) row grouped by expert, expert e's segment starting
  at poff[e] (a multiple of 64, zero rows in the padding).  Forward gate|up (gemm_moe) -> SiLU*mul ->
  down (gemm_moe).  Backward: input gradients through the per-expert transposed weights (gemm_moe), and
  the weight gradients dW_e = dY_e^T X_e of every expert at once by the K-grouped GEMM (gemm_kgroup over
  the transposed / shuffled-transposed slot arrays), accumulated straight into the stacks' GradAcc
  buffers (plain store on the first micro-batch of a step, in place after)."""

  @staticmethod
  def forward(ctx, xs, poff, max_rows, sgu, sdown, agu, adown):
    gu = _grouped(xs, sgu.ws, poff, max_rows)  # [P, 2F]
    act = torch.empty(xs.shape[0], gu.shape[1] // 2, dtype=torch.bfloat16, device=xs.device)
    require().silu_mul(gu, act, False)
    y = _grouped(act, sdown.ws, poff, max_rows)  # [P, D]
    ctx.save_for_backward(xs, poff, gu, act)
    ctx.max_rows, ctx.sgu, ctx.sdown, ctx.agu, ctx.adown = max_rows, sgu, sdown, agu, adown
    return y

  @staticmethod
  def backward(ctx, dy):
    xs, poff, gu, act = ctx.saved_tensors
    dy = dy.contiguous()
    C = require()
    d_act = _grouped(dy, ctx.sdown.wts, poff, ctx.max_rows)  # [P, F]
    _kgroup_acc(relayout(dy, 2), relayout(act, 1), ctx.adown, poff)  # dW_down[e] = dy_e^T act_e
    d_gu = torch.empty_like(gu)
    C.silu_mul_bwd(gu, d_act, d_gu)
    dxs = _grouped(d_gu, ctx.sgu.wts, poff, ctx.max_rows)  # [P, D]
    _kgroup_acc(relayout(d_gu, 2), relayout(xs, 1), ctx.agu, poff)  # dW_gu[e] = d_gu_e^T xs_e
    return dxs, None, None, None, None, None, None


def _kgroup_acc(at, bts, acc, poff):
  fresh = acc.fresh
  require().gemm_kgroup(at, bts, acc.buf, poff, not fresh)
  acc.fresh = False
  if acc.cb is not None:
    acc.cb()


def grouped_experts(xs, poff, max_rows, sgu, sdown, agu, adown):
  return GroupedExpertsFn.apply(xs, poff, max_rows, sgu, sdown, agu, adown)


class RouterFn(torch.autograd.Function):
  """MoE router scores in fp32, logits [T, E] = x . W^T, on the kernel library: forward the router_logits
  kernel (fp32 accumulation of bf16 inputs, as the serving path), backward two own GEMMs on the tiles with the
  gradient rounded to bf16 and E zero-padded to 128 (E x D is small): dX = dL . W (shuffle(W^T) rebuilt per
  call) and dW = dL^T . X (T zero-padded to 128 rows as in own_dw)."""

  @staticmethod
  def forward(ctx, x, w):
    T, E = x.shape[0], w.shape[0]
    out = torch.empty(T, E, dtype=torch.float32, device=x.device)
    require().router_logits(x, w, out)
    ctx.save_for_backward(x, w)
    return out

  @staticmethod
  def backward(ctx, dl):
    from ..ops.linear import linear
    x, w = ctx.saved_tensors
    E, D = w.shape
    Ep = -(-E // 128) * 128
    dlb = dl.to(torch.bfloat16)
    a = torch.zeros(dlb.shape[0], Ep, dtype=torch.bfloat16, device=x.device)
    a[:, :E] = dlb
    wp = torch.zeros(Ep, D, dtype=torch.bfloat16, device=x.device)
    wp[:E] = w
    dx = linear(a, relayout(wp, 1))  # [T, D] = dL . W
    dw = linear(relayout(pad_rows(a), 2), relayout(pad_rows(x), 1))[:E]  # [E, D] = dL^T . X (Ep rows, E kept)
    return dx, dw.to(w.dtype)


def router_ok(x: torch.Tensor, w: torch.Tensor) -> bool:
  E, D = w.shape
  return x.is_cuda and x.dtype == w.dtype == torch.bfloat16 and D % 128 == 0 and \
      (E in (4, 8, 16) or (E in (32, 64, 128, 160, 256) and D % 512 == 0))  # launch_router_logits' cases


def router_logits(x, w):
  """fp32 router logits [T, E] with autograd to x and w (RouterFn on the GPU, fp32 torch on the CPU)."""
  if router_ok(x, w):
    return RouterFn.apply(x.contiguous(), w)
  return x.float() @ w.float().t()


class LmHeadCEFn(torch.autograd.Function):
  """sum_t w_t CE(xn_t . head^T, y_t) without materialising [T, V] logits: row chunks of `chunk`
  tokens; per chunk the fp32 logits come from the own GEMM, ce_fwd / ce_bwd give the loss and dlogits (bf16),
  and -- the loss being the last op, its upstream gradient a scalar -- dX_c = dlogits_c . head and
  dHead += dlogits_c^T . X_c are formed right there, so the backward only scales the saved gradients.
  Peak memory: one [chunk, V] fp32 logits block + its bf16 gradient.  With a GradAcc `acc` (an untied head) the
  dHead GEMMs accumulate straight into it through own_dw -- on the weight-gradient side stream, beside the rest of
  the backward -- and the head gets no autograd gradient (no [V, D] add per micro-batch)."""

  @staticmethod
  def forward(ctx, xn, head, tw, targets, weights, chunk, acc=None):
    from ..ops.linear import linear
    T0 = xn.shape[0]
    # ragged token counts: zero rows with ignored targets (their dlogits rows are zero) up to a multiple of 128,
    # so every chunk's dHead GEMM runs on the tiles
    assert chunk % 128 == 0, chunk
    xn, targets, weights = pad_rows(xn), pad_rows(targets, value=-1), pad_rows(weights)
    T, D = xn.shape
    C = require()
    dxn = torch.empty_like(xn)
    dhead = torch.empty(head.shape if acc is None else (0,), dtype=torch.bfloat16, device=xn.device)
    total = torch.zeros((), dtype=torch.float32, device=xn.device)
    for i, r0 in enumerate(range(0, T, chunk)):
      r1 = min(T, r0 + chunk)
      xc = xn[r0:r1]
      logits = linear(xc, tw.ws, out_dtype=torch.float32)  # [c, V]
      loss = torch.empty(r1 - r0, dtype=torch.float32, device=xn.device)
      lse = torch.empty_like(loss)
      tc = targets[r0:r1].contiguous()
      C.ce_fwd(logits, tc, loss, lse)
      wc = weights[r0:r1].float().contiguous()
      total += (loss * wc).sum()
      dl = torch.empty(logits.shape, dtype=torch.bfloat16, device=xn.device)
      C.ce_bwd(logits, tc, lse, wc, dl)
      del logits
      linear(dl, tw.wts, out=dxn[r0:r1])
      if acc is not None:
        own_dw(dl, xc, acc, cb=False)
        continue
      if dw_tn(dl, xc, dhead, i > 0):
        continue
      dlt, xts = relayout(dl, 2), relayout(xc, 1)  # dlogits^T [V, c], shuffle(X_c^T) [D, c]
      if i == 0:
        linear(dlt, xts, out=dhead)
      else:
        linear(dlt, xts, residual=dhead, epi="resid", out=dhead)
    if acc is not None and acc.cb is not None:
      acc.cb()
    ctx.acc = acc
    ctx.save_for_backward(dxn[:T0], dhead)
    return total

  @staticmethod
  def backward(ctx, g):
    dxn, dhead = ctx.saved_tensors
    if not (isinstance(g, torch.Tensor) and g.numel() == 1 and float(g) == 1.0):
      if ctx.acc is not None:
        raise RuntimeError("a scaled loss cannot reach the head gradient already accumulated in its GradAcc")
      dxn, dhead = dxn * g.to(dxn.dtype), dhead * g.to(dhead.dtype)
    return dxn, (None if ctx.acc is not None else dhead), None, None, None, None, None


def lm_head_ce(xn, head, tw, targets, weights, chunk: int = 1024, acc=None):
  """xn [T, D] bf16, head [V, D] (its TrainWeight tw), targets [T] int32 (< 0 ignored), weights [T] fp32;
  `acc`: the head's GradAcc (then the head gradient is accumulated there, not returned)."""
  return LmHeadCEFn.apply(xn.contiguous(), head, tw, targets, weights, chunk, acc)


class QKVSplitFn(torch.autograd.Function):
  """Fused-QKV projection output [T, (H + 2 Hkv) Dh] -> q, k (contiguous copies) and v (a row-strided view).
  The backward concatenates dq | dk | dv once; autograd's slice backwards would zero-fill three full-size
  gradients, copy each slice in and add them (3 fills + 3 copies + 2 adds per layer and micro-batch)."""

  @staticmethod
  def forward(ctx, qkv, nq, nk):
    ctx.widths = (nq, nk, qkv.shape[1] - nq - nk)
    return qkv[:, :nq].contiguous(), qkv[:, nq:nq + nk].contiguous(), qkv[:, nq + nk:]

  @staticmethod
  def backward(ctx, dq, dk, dv):
    ref = next(g for g in (dq, dk, dv) if g is not None)
    parts = [g if g is not None else ref.new_zeros(ref.shape[0], w) for g, w in zip((dq, dk, dv), ctx.widths)]
    return torch.cat(parts, dim=1), None, None


def qkv_split(qkv, nq, nk):
  return QKVSplitFn.apply(qkv, nq, nk)


class QKVRopeFn(torch.autograd.Function):
  """Fused-QKV projection output [T, (H + 2 Hkv) Dh] -> rope(q), rope(k) (contiguous) and v (a row-strided view),
  in two rope_apply launches that read q / k straight out of the qkv rows (QKVSplitFn + RopeFn made contiguous
  copies first).  The backward writes the inverse rotations of dq / dk and dv straight into the slices of one
  dqkv buffer instead of rotating into temporaries and concatenating."""

  @staticmethod
  def forward(ctx, qkv, pos, cos_sin, H, Hkv, Dh):
    C = require()
    T, nq, nk = qkv.shape[0], H * Dh, Hkv * Dh
    ctx.save_for_backward(pos, cos_sin)
    ctx.dims = (H, Hkv, Dh, qkv.shape[1])
    q = torch.empty(T, nq, dtype=qkv.dtype, device=qkv.device)
    k = torch.empty(T, nk, dtype=qkv.dtype, device=qkv.device)
    C.rope_apply(qkv[:, :nq], q, pos, cos_sin, int(H), int(Dh), False)
    C.rope_apply(qkv[:, nq:nq + nk], k, pos, cos_sin, int(Hkv), int(Dh), False)
    return q, k, qkv[:, nq + nk:]

  @staticmethod
  def backward(ctx, dq, dk, dv):
    C = require()
    pos, cos_sin = ctx.saved_tensors
    H, Hkv, Dh, W = ctx.dims
    nq, nk = H * Dh, Hkv * Dh
    ref_t = next(g for g in (dq, dk, dv) if g is not None)
    dqkv = torch.empty(ref_t.shape[0], W, dtype=ref_t.dtype, device=ref_t.device)
    for g, lo, n, nh in ((dq, 0, nq, H), (dk, nq, nk, Hkv)):
      if g is None:
        dqkv[:, lo:lo + n].zero_()
      else:
        C.rope_apply(g.contiguous(), dqkv[:, lo:lo + n], pos, cos_sin, int(nh), int(Dh), True)
    if dv is None:
      dqkv[:, nq + nk:].zero_()
    else:
      dqkv[:, nq + nk:].copy_(dv)
    return dqkv, None, None, None, None, None


class QKVAttentionFn(torch.autograd.Function):
  """Fused-QKV projection output [T, (H + 2 Hkv) Dh] -> causal GQA attention of (rope(q), rope(k), v): QKVRopeFn +
  AttentionFn in one node, so q and k rotate in ONE rope_apply launch (their heads are adjacent columns) into one
  [T, (H + Hkv) Dh] buffer the attention reads as two strided views, and the backward writes dq / dk side by side
  (one inverse rope_apply into the dqkv rows) and dv straight into its dqkv slice (no copy)."""

  @staticmethod
  def forward(ctx, qkv, pos, cos_sin, B, L, H, Hkv, Dh):
    C = require()
    scale = Dh ** -0.5
    Lp = -(-L // 64) * 64
    T, nq, nk = qkv.shape[0], H * Dh, Hkv * Dh
    qk = torch.empty(T, nq + nk, dtype=qkv.dtype, device=qkv.device)
    C.rope_apply(qkv[:, :nq + nk], qk, pos, cos_sin, int(H + Hkv), int(Dh), False)
    q, k, v = qk[:, :nq], qk[:, nq:], qkv[:, nq + nk:]
    o = torch.empty(T, nq, dtype=qkv.dtype, device=qkv.device)
    lse2 = torch.empty(B * H * L, dtype=torch.float32, device=qkv.device)
    vt = _transposed(C, v, B, L, Lp, Hkv, Dh)
    C.attn_train_fwd(q, k, vt, o, lse2, B, L, Lp, H, Hkv, Dh, scale, True)
    ctx.save_for_backward(qk, qkv, o, lse2, pos, cos_sin)
    ctx.dims = (B, L, Lp, H, Hkv, Dh, scale)
    return o

  @staticmethod
  def backward(ctx, do):
    C = require()
    qk, qkv, o, lse2, pos, cos_sin = ctx.saved_tensors
    B, L, Lp, H, Hkv, Dh, scale = ctx.dims
    T, nq, nk = qk.shape[0], H * Dh, Hkv * Dh
    do = do.contiguous().to(qk.dtype)
    dqkv = torch.empty(T, qkv.shape[1], dtype=qk.dtype, device=qk.device)
    dqk = torch.empty_like(qk)
    delta = torch.empty_like(lse2)
    ws = torch.empty(2 * H * B * L * Dh, dtype=torch.float32, device=qk.device)  # per-query-head dK/dV partials
    C.attn_train_bwd(qk[:, :nq], qk[:, nq:], qkv[:, nq + nk:], o, do, lse2, delta, dqk[:, :nq], dqk[:, nq:],
                     dqkv[:, nq + nk:], ws, B, L, Lp, H, Hkv, Dh, scale)
    C.rope_apply(dqk, dqkv[:, :nq + nk], pos, cos_sin, int(H + Hkv), int(Dh), True)
    return dqkv, None, None, None, None, None, None, None


def qkv_attention(qkv, pos, cos_sin, B, L, H, Hkv, Dh):
  """Causal GQA attention of a fused-QKV projection output with RoPE on q / k (QKVAttentionFn on the GPU)."""
  if _gpu(qkv) and qkv.stride(1) == 1 and Dh in (64, 128):
    return QKVAttentionFn.apply(qkv, pos, cos_sin, B, L, H, Hkv, Dh)
  q, k, v = qkv_rope(qkv, pos, cos_sin, H, Hkv, Dh)
  return attention(q, k, v, B, L, H, Hkv, Dh)


def qkv_rope(qkv, pos, cos_sin, H, Hkv, Dh):
  """(rope(q), rope(k), v) of a fused-QKV projection output (QKVRopeFn on the GPU)."""
  if _gpu(qkv) and qkv.stride(1) == 1:
    return QKVRopeFn.apply(qkv, pos, cos_sin, H, Hkv, Dh)
  q, k, v = qkv_split(qkv, H * Dh, Hkv * Dh)
  return rope(q, pos, cos_sin, H, Dh), rope(k, pos, cos_sin, Hkv, Dh), v

"""Autograd functions over the gfx950 kernel library (fp32 torch math on CPU tensors).

  RMSNormFn    forward rmsnorm kernel, backward rmsnorm_bwd kernel (dx + fp32 dw reduction)
  SiluMulFn    [gate | up] -> silu(gate) * up, backward silu_mul_bwd kernel
  RopeFn       rotate-half RoPE; backward = the inverse rotation (same kernel, sin negated)
  CrossEntropyFn  per-row loss with ignore (-100) and per-row weights; forward ce_fwd, backward ce_bwd
Projections use torch.matmul (hipBLASLt) and attention uses torch SDPA in the training path.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ..ops import reference as ref
from ..ops._ext import require


def _gpu(t: torch.Tensor) -> bool:
  return t.is_cuda


class RMSNormFn(torch.autograd.Function):
  @staticmethod
  def forward(ctx, x, w, eps):
    ctx.eps = eps
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
      dw = torch.zeros(w.numel(), dtype=torch.float32, device=x.device)
      require().rmsnorm_bwd(x.contiguous(), w, dy.contiguous().to(x.dtype), dx, dw, float(ctx.eps))
      return dx, dw.to(w.dtype), None
    with torch.enable_grad():
      xr = x.detach().float().requires_grad_()
      wr = w.detach().float().requires_grad_()
      y = xr * torch.rsqrt(xr.pow(2).mean(-1, keepdim=True) + ctx.eps) * wr
      y.backward(dy.float())
    return xr.grad.to(x.dtype), wr.grad.to(w.dtype), None


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


def rmsnorm(x, w, eps):
  return RMSNormFn.apply(x, w, eps)


def silu_mul(gu):
  return SiluMulFn.apply(gu)


def rope(x, pos, cos_sin, nh, Dh):
  return RopeFn.apply(x, pos, cos_sin, nh, Dh)


def cross_entropy(logits, targets, weights):
  return CrossEntropyFn.apply(logits, targets, weights)

"""Projection dispatch: hand-written fused MFMA GEMM vs hipBLASLt + epilogue kernel, per shape.

Every projection of the transformer goes through `linear()`.  Two implementations exist on GPU:

  hip   the library's own MFMA GEMM with the epilogue fused (bias / residual add / SiLU*mul)
  blas  hipBLASLt (torch.matmul / addmm) for the plain GEMM + the library's epilogue kernel

`GemmPolicy` picks per (M, N, K, epilogue) by timing both once on first use (eager, before any HIP
graph capture) unless XOT_GEMM=hip|blas forces one.  Decisions are kept per process and can be
dumped/loaded as JSON (`XOT_GEMM_TABLE`).  CPU tensors use the fp32 reference.
"""
from __future__ import annotations

import json
import os
from typing import Dict, Tuple

import torch

from . import kernels as K


def _m_bucket(M: int) -> int:
  b = 1
  while b < M:
    b *= 2
  return b


class GemmPolicy:
  def __init__(self):
    self.mode = os.environ.get("XOT_GEMM", "auto")
    self.table: Dict[Tuple[int, int, int, str, bool], str] = {}
    path = os.environ.get("XOT_GEMM_TABLE")
    if path and os.path.exists(path):
      with open(path) as f:
        for k, v in json.load(f).items():
          m, n, k_, e, b = k.split(",")
          self.table[(int(m), int(n), int(k_), e, b == "1")] = v
    self.capturing = False

  def dump(self, path: str):
    with open(path, "w") as f:
      json.dump({f"{m},{n},{k},{e},{int(b)}": v for (m, n, k, e, b), v in self.table.items()}, f, indent=1)

  def choose(self, x, w, bias, residual, epi, out_dtype) -> str:
    if self.mode in ("hip", "blas"):
      return self.mode
    M, Kd = x.shape
    N = w.shape[0]
    key = (_m_bucket(M), N, Kd, epi, bias is not None)
    got = self.table.get(key)
    if got is not None:
      return got
    if self.capturing or torch.cuda.is_current_stream_capturing():
      return "hip"  # never time inside a capture; default to the fused kernel
    got = self._tune(x, w, bias, residual, epi, out_dtype)
    self.table[key] = got
    return got

  def _tune(self, x, w, bias, residual, epi, out_dtype) -> str:
    times = {}
    res_copy = residual.clone() if residual is not None else None
    for impl in ("hip", "blas"):
      try:
        fn = lambda: _run(impl, x, w, bias, res_copy, epi, None, out_dtype)  # noqa: E731
        fn()
        torch.cuda.synchronize()
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        best = float("inf")
        for _ in range(3):
          st.record()
          for _ in range(3):
            fn()
          en.record()
          en.synchronize()
          best = min(best, st.elapsed_time(en))
        times[impl] = best
      except RuntimeError:
        times[impl] = float("inf")
    return min(times, key=times.get)


policy = GemmPolicy()


def _run(impl, x, w, bias, residual, epi, out, out_dtype):
  if impl == "hip":
    return K.gemm(x, w, bias=bias, residual=residual, epi=epi, out=out, out_dtype=out_dtype)
  M, N = x.shape[0], w.shape[0]
  if epi == "silu":
    tmp = torch.matmul(x, w.t())
    if bias is not None:
      tmp += bias
    return K.silu_mul(tmp, out=out, interleaved16=True)
  if epi == "resid":
    if out is not None and out.data_ptr() == residual.data_ptr():
      out.addmm_(x, w.t())  # in-place residual stream update
    else:
      if out is None:
        out = torch.empty(M, N, dtype=out_dtype or x.dtype, device=x.device)
      torch.addmm(residual, x, w.t(), out=out)
    if bias is not None:
      out += bias
    return out
  dt = out_dtype or (out.dtype if out is not None else x.dtype)
  if dt == x.dtype:
    if out is None:
      out = torch.empty(M, N, dtype=dt, device=x.device)
    if bias is not None:
      torch.addmm(bias, x, w.t(), out=out)
    else:
      torch.matmul(x, w.t(), out=out)
    return out
  y = torch.matmul(x, w.t()).to(dt)
  if bias is not None:
    y += bias.to(dt)
  if out is not None:
    out.copy_(y)
    return out
  return y


def linear(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor | None = None, residual: torch.Tensor | None = None,
           epi: str = "none", out: torch.Tensor | None = None, out_dtype: torch.dtype | None = None) -> torch.Tensor:
  if not x.is_cuda:
    return K.gemm(x, w, bias=bias, residual=residual, epi=epi, out=out, out_dtype=out_dtype)
  impl = policy.choose(x, w, bias, residual, epi, out_dtype or (out.dtype if out is not None else x.dtype))
  return _run(impl, x, w, bias, residual, epi, out, out_dtype)

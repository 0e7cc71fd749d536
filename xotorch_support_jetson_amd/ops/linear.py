"""Projection dispatch for the transformer: y = x @ W.T with a fused epilogue.

GPU weights of the decode path are stored PRE-SHUFFLED (ops.weights_layout.shuffle_for_stream;
tagged `w.xot_layout == "stream"`).  Per call:

  M <= 128 (decode, small prefill chunks)
        gemm_stream: the library's weight-streaming MFMA GEMM on the shuffled layout (1 KB coalesced
        weight loads per wave instruction, X shared through swizzled LDS) with the epilogue fused
        (bias / residual add / SiLU*mul).  (ntw, split-K) is autotuned per shape on first use.
  128 < M <= 256
        the same kernel over 128-row slices (weights re-read once more, still cheaper than a copy)
  M > 256 (prefill)
        unshuffle the weight into a per-device scratch buffer and run hipBLASLt (torch.matmul/addmm)
        + the library's epilogue kernel; the copy is ~5 % of a long prefill GEMM.

Row-major (un-shuffled) GPU weights use the GemmPolicy (own skinny/tiled kernels vs hipBLASLt, timed
once per shape).  CPU tensors use the fp32 reference.  Autotuning never runs inside a HIP-graph
capture (the runner warms every captured shape up eagerly first).
"""
from __future__ import annotations

import json
import os
from typing import Dict, Tuple

import torch

from . import kernels as K
from ._ext import require
from .weights_layout import can_shuffle, shuffle_for_stream, unshuffle_from_stream


def _m_bucket(M: int) -> int:
  b = 1
  while b < M:
    b *= 2
  return b


def layout_of(w: torch.Tensor) -> str:
  return getattr(w, "xot_layout", "rowmajor")


def to_stream_layout(w: torch.Tensor) -> torch.Tensor:
  """Shuffled copy of a row-major [N, K] GPU weight, tagged for the stream GEMM."""
  if not (w.is_cuda and can_shuffle(w)):
    return w
  s = shuffle_for_stream(w)
  s.xot_layout = "stream"
  return s


def to_rowmajor(w: torch.Tensor) -> torch.Tensor:
  return unshuffle_from_stream(w) if layout_of(w) == "stream" else w


# ------------------------------------------------------------------ per-device scratch
class _Scratch:
  def __init__(self):
    self.ws: Dict[int, torch.Tensor] = {}
    self.dense: Dict[int, torch.Tensor] = {}

  def splitk(self, device, n: int) -> torch.Tensor:
    idx = device.index or 0
    t = self.ws.get(idx)
    if t is None or t.numel() < n:
      if torch.cuda.is_current_stream_capturing():
        raise RuntimeError("split-K workspace must be sized before graph capture")
      t = torch.empty(max(n, 1 << 20), dtype=torch.float32, device=device)
      self.ws[idx] = t
    return t

  def dense_weight(self, w: torch.Tensor) -> torch.Tensor:
    """Row-major copy of a shuffled weight in a reusable buffer (prefill path)."""
    idx = w.device.index or 0
    n = w.numel()
    t = self.dense.get(idx)
    if t is None or t.numel() < n:
      t = torch.empty(n, dtype=w.dtype, device=w.device)
      self.dense[idx] = t
    N, Kd = w.shape
    v = t[:n].view(N // 16, 16, Kd // 128, 4, 4, 8)
    v.copy_(w.view(N // 16, Kd // 128, 4, 4, 16, 8).permute(0, 4, 1, 3, 2, 5))
    return t[:n].view(N, Kd)


scratch = _Scratch()


class GemmPolicy:
  def __init__(self):
    self.mode = os.environ.get("XOT_GEMM", "auto")
    self.table: Dict[Tuple, object] = {}
    path = os.environ.get("XOT_GEMM_TABLE")
    if path and os.path.exists(path):
      with open(path) as f:
        for k, v in json.load(f).items():
          self.table[tuple(json.loads(k))] = tuple(v) if isinstance(v, list) else v
    self.capturing = False

  def dump(self, path: str):
    with open(path, "w") as f:
      json.dump({json.dumps(list(k)): v for k, v in self.table.items()}, f, indent=1)

  @staticmethod
  def _time(fn) -> float:
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
    return best

  def _no_tuning(self) -> bool:
    return self.capturing or torch.cuda.is_current_stream_capturing()

  # ---------------------------------------------------------------- row-major weights
  def choose(self, x, w, bias, residual, epi, out_dtype) -> str:
    if self.mode in ("hip", "blas"):
      return self.mode
    M, Kd = x.shape
    key = ("rm", _m_bucket(M), w.shape[0], Kd, epi, bias is not None)
    got = self.table.get(key)
    if got is not None:
      return got
    if self._no_tuning():
      return "hip"
    times = {}
    res_copy = residual.clone() if residual is not None else None
    for impl in ("hip", "blas"):
      try:
        times[impl] = self._time(lambda: _run_rowmajor(impl, x, w, bias, res_copy, epi, None, out_dtype))
      except RuntimeError:
        times[impl] = float("inf")
    got = min(times, key=times.get)
    self.table[key] = got
    return got

  # ---------------------------------------------------------------- shuffled weights
  def stream_cfg(self, x, w, bias, residual, epi, out_dtype) -> Tuple[int, int]:
    M, Kd = x.shape
    N = w.shape[0]
    key = ("st", _m_bucket(M), N, Kd, epi, bias is not None, str(out_dtype))
    got = self.table.get(key)
    if got is not None:
      return got
    cands = []
    for ntw in ((2, 4) if epi == "silu" else (1, 2, 4)):
      if N % (64 * ntw) or (ntw == 4 and M <= 32):
        continue
      for S in (1, 2, 4, 8):
        if Kd % (S * 256) == 0 and (N // (64 * ntw)) * S <= 4096:
          cands.append((ntw, S))
    if not cands:
      raise RuntimeError(f"no stream-GEMM configuration for N={N} K={Kd}")
    if self._no_tuning():
      return self._heuristic(M, N, cands)
    scratch.splitk(x.device, 8 * 128 * N)
    y = torch.empty(M, N // 2 if epi == "silu" else N, dtype=out_dtype, device=x.device)
    times = {}
    for cfg in cands:
      try:
        times[cfg] = self._time(lambda: _stream_call(x, w, bias, residual, epi, y, cfg))
      except RuntimeError:
        pass
    got = min(times, key=times.get) if times else cands[0]
    self.table[key] = got
    return got

  @staticmethod
  def _heuristic(M, N, cands):
    # enough workgroups to cover 256 CUs a few times
    best = None
    for ntw, S in cands:
      wg = (N // (64 * ntw)) * S
      score = abs(wg - 768)
      if best is None or score < best[0]:
        best = (score, (ntw, S))
    return best[1]


policy = GemmPolicy()


def _stream_call(x, w, bias, residual, epi, out, cfg):
  ntw, S = cfg
  M, N = x.shape[0], w.shape[0]
  ws = scratch.splitk(x.device, S * M * N) if S > 1 else None
  require().gemm_stream(x, w, out, bias, residual, ws, K.EPI[epi], ntw, S, True)
  return out


def _run_rowmajor(impl, x, w, bias, residual, epi, out, out_dtype):
  if impl == "hip":
    return K.gemm(x, w, bias=bias, residual=residual, epi=epi, out=out, out_dtype=out_dtype)
  return _blas(x, w, bias, residual, epi, out, out_dtype)


def _blas(x, w, bias, residual, epi, out, out_dtype):
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
    return K.gemm(x, to_rowmajor(w), bias=bias, residual=residual, epi=epi, out=out, out_dtype=out_dtype)
  dt = out_dtype or (out.dtype if out is not None else x.dtype)
  M, N = x.shape[0], w.shape[0]
  if layout_of(w) != "stream":
    impl = policy.choose(x, w, bias, residual, epi, dt)
    return _run_rowmajor(impl, x, w, bias, residual, epi, out, out_dtype)
  if M > 256:
    return _blas(x, scratch.dense_weight(w), bias, residual, epi, out, out_dtype)
  if out is None:
    out = torch.empty(M, N // 2 if epi == "silu" else N, dtype=dt, device=x.device)
  if x.stride(1) != 1:
    x = x.contiguous()
  for lo in range(0, M, 128):  # rows are independent: 128-row slices share one tuned config
    hi = min(M, lo + 128)
    xs, ys = x[lo:hi], out[lo:hi]
    rs = residual[lo:hi] if residual is not None else None
    cfg = policy.stream_cfg(xs, w, bias, rs, epi, dt)
    _stream_call(xs, w, bias, rs, epi, ys, cfg)
  return out

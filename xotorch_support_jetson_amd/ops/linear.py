"""Projection dispatch for the transformer: y = x @ W.T with a fused epilogue.

GPU weights are stored PRE-SHUFFLED (ops.weights_layout.shuffle_for_stream; tagged
`w.xot_layout == "stream"`): 16-row x 32-k MFMA B-fragment blocks, 1 KB each.  Two library kernels
consume that layout, both with the epilogue fused (bias / residual add / SiLU*mul):

  gemm_stream  decode-shaped M: weight-streaming MFMA GEMM (1 KB coalesced weight loads per wave
               instruction straight to registers, X shared through swizzled LDS, optional split-K).
  gemm_big     compute-bound M (large decode batches, prefill chunks): 256 x {256,128} x 64 tiles,
               both operands staged by LDS-DMA, 8 waves, XCD-aware tile order, optional split-K.
No vendor GEMM runs on a shuffled weight: at prefill sizes gemm_big matches hipBLASLt once the weight
copy the library would need is counted (profiles/r3/bench_gemm_sk.json), so there is no un-shuffle path.

The configuration ((kernel, ntw|bn, split-K) per M bucket and shape) is chosen by cold-cache timing on
first use; inside a HIP-graph capture a heuristic stands in (the runner warms every captured shape up
eagerly first, so the timed choice is normally cached).  Row-major GPU weights use the GemmPolicy
(own skinny/tiled kernels vs hipBLASLt).  CPU tensors use the fp32 reference.
"""
from __future__ import annotations

import json
import os
import sys
from typing import Dict, Tuple

import torch

from . import kernels as K
from ._ext import require
from .weights_layout import (can_shuffle, dequant_stream8, dequant_stream8_to_stream, quantize_fp8_rows,
                             shuffle_for_stream, shuffle_for_stream8, unshuffle_from_stream)


# (A stream-K kernel -- persistent 256 x 256 workgroups, k steps dealt evenly -- won the isolated timing of gate/up
# at M = 512 but fetched ~37 % more bytes from beyond L2 than the ping-pong tile and ran the whole decode step 0.9 %
# slower under the board power cap, 81.64 vs 80.95 ms, profiles/r4/tuner/; removed in round 6.)
# XOT_GEMM_PP2=0: leave the two-phase ping-pong tile (code 2256) out of the candidates
PP2 = os.environ.get("XOT_GEMM_PP2", "1") == "1"
# XOT_GEMM_W4=0: leave the four-wave 256 x 256 tile (code 4256) out of the candidates
W4 = os.environ.get("XOT_GEMM_W4", "1") == "1"
# rows from which the four-wave tile is preferred over the two-phase ping-pong within TIE (tall prefill / training
# GEMMs: it reads a third less LDS per FLOP and has ~6 us less fixed cost per tile, profiles/r5/gemm_w4/); below
# it the ping-pong tile, the measured in-step winner at the decode batches, keeps the preference
W4_PREF_M = int(os.environ.get("XOT_GEMM_W4_PREF_M", "2048"))
# tall GEMMs take the four-wave tile without a timing pass (see shuffled_cfg; tests switch it off)
TALL_FIXED = True
# XOT_GEMM_BLAS=1: time hipBLASLt among the candidates for row-major weights (off: the kernel library only)
BLAS_CAND = os.environ.get("XOT_GEMM_BLAS", "0") == "1"
# largest M for which the stream GEMM is a candidate (above it only gemm_big is timed)
STREAM_MAX_M = int(os.environ.get("XOT_STREAM_MAX_M", "512"))
# smallest M for which gemm_big is a candidate
BIG_MIN_M = int(os.environ.get("XOT_BIG_MIN_M", "65"))


def _m_bucket(M: int) -> int:
  """Tuning-table key of a row count: powers of two up to 256, then multiples of 64 up to 1024 (the decode
  batch buckets 320 / 384 / 448 tile differently from 512: row tiles of 160 / 192 / 224), then powers of two."""
  if 256 < M <= 1024:
    return -(-M // 64) * 64
  b = 1
  while b < M:
    b *= 2
  return b


def big_row_tile(M: int) -> int:
  """Row tile of the large-M GEMM for M rows: 256, or -- when ceil(M / 256) tiles of 256 would carry 32 or more
  padding rows -- the smallest multiple of 32 (>= 160) that covers M in that many tiles."""
  n = -(-M // 256)
  bm = max(160, -(-M // (32 * n)) * 32)
  return bm if bm < 256 else 256


def tile_width(code: int) -> int:
  """Columns of a gemm_big tile code (BN, 1256 / 2256 = 256 on the four- / two-phase ping-pong, + 10000 x BM)."""
  return code % 1000


def tile_rows(code: int) -> int:
  return code // 10000 or 256


def layout_of(w: torch.Tensor) -> str:
  return getattr(w, "xot_layout", "rowmajor")


def to_stream_layout(w: torch.Tensor) -> torch.Tensor:
  """Shuffled copy of a row-major [N, K] GPU weight, tagged for the stream GEMM."""
  if not (w.is_cuda and can_shuffle(w)):
    return w
  s = shuffle_for_stream(w)
  s.xot_layout = "stream"
  return s


def to_stream8_layout(w: torch.Tensor) -> torch.Tensor:
  """Weight-only FP8 copy of a row-major [N, K] GPU weight: shuffled e4m3 bytes tagged "stream8", the
  per-row fp32 scales in `.xot_scale`."""
  if not (w.is_cuda and can_shuffle(w)):
    return w
  q, sc = quantize_fp8_rows(w)
  s = shuffle_for_stream8(q)
  s.xot_layout = "stream8"
  s.xot_scale = sc
  return s


def to_rowmajor(w: torch.Tensor) -> torch.Tensor:
  if layout_of(w) == "stream8":
    return dequant_stream8(w, w.xot_scale)
  return unshuffle_from_stream(w) if layout_of(w) == "stream" else w


# ------------------------------------------------------------------ per-device scratch
class _Scratch:
  """Per-device split-K slabs shared by every GEMM call.  A buffer that has to grow is replaced, but the old one is
  kept alive: HIP graphs captured earlier (decode graphs of other batch buckets) hold its address, and replaying
  them into a freed block would corrupt whatever the caching allocator put there next (a serving run that captured
  bucket 1, then grew the slabs for bucket 64, faulted exactly that way)."""

  def __init__(self):
    self.ws: Dict[int, torch.Tensor] = {}
    self.retired: list = []

  def splitk(self, device, n: int, slot: int = 0) -> torch.Tensor:
    """slot 1 holds the slabs of a residual projection whose reduce is deferred into the next GEMM (PendingNorm),
    which writes its own slabs to slot 0 while it still reads slot 1."""
    key = (device.index or 0, slot)
    t = self.ws.get(key)
    if t is None or t.numel() < n:
      if torch.cuda.is_current_stream_capturing():
        raise RuntimeError("split-K workspace must be sized before graph capture")
      if t is not None:
        self.retired.append(t)
      t = torch.empty(max(n, 1 << 20, 2 * (t.numel() if t is not None else 0)), dtype=torch.float32, device=device)
      self.ws[key] = t
    return t


scratch = _Scratch()


def _default_table_path():
  """Where tuned GEMM choices persist: per GPU model and kernel-library build (a rebuilt library may rank
  the kernels differently), under XOT_HOME.  XOT_GEMM_TABLE overrides; XOT_GEMM_TABLE=off disables."""
  env = os.environ.get("XOT_GEMM_TABLE")
  if env:
    return None if env == "off" else env
  try:
    if not torch.cuda.is_available():
      return None
    from .. import _C
    st = os.stat(_C.__file__)
    dev = torch.cuda.get_device_name(torch.cuda.current_device()).replace(" ", "_").replace("/", "_")
    from ..helpers import xot_home
    # settings that change the candidate sets are part of the name, so a table never answers for another
    tag = (f"{os.environ.get('XOT_GEMM', 'auto')}-{STREAM_MAX_M}-{BIG_MIN_M}-{SLAB_TBPS:g}"
           f"{'-blas' if BLAS_CAND else ''}-t{TIE:g}-x{TIE_X:g}{'' if PP2 else '-nopp2'}")
    return str(xot_home() / "gemm" / f"{dev}-{st.st_size:x}-{int(st.st_mtime):x}-{tag}.json")
  except Exception:  # noqa: BLE001 - no table then; tuning still works in memory
    return None


# Seed table: the headline decode step's picks (ops/gemm_seed_mi355x.json), tuned on MI355X over rounds 4-6 and
# stable there, loaded under the box's own table so a fresh box runs them without re-timing in a noisy warmup.
# XOT_GEMM_SEED=0 (or XOT_GEMM_TABLE=off, or another GPU): tuned in-process like every other shape.
SEED_TABLE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "gemm_seed_mi355x.json")


def _seed_table_path():
  if os.environ.get("XOT_GEMM_SEED", "1") == "0" or os.environ.get("XOT_GEMM_TABLE") == "off":
    return None
  try:
    if not torch.cuda.is_available():
      return None
    i = torch.cuda.current_device()
    arch = getattr(torch.cuda.get_device_properties(i), "gcnArchName", "")
    if not (arch.startswith("gfx950") or "MI355" in torch.cuda.get_device_name(i)):  # CDNA4 (gfx950) only
      return None
  except Exception:  # noqa: BLE001
    return None
  return SEED_TABLE if os.path.exists(SEED_TABLE) else None


class GemmPolicy:
  """GEMM implementation choice per (layout, M bucket, N, K, epilogue, ...), cold-cache timed on first use.
  Choices persist in a JSON table (see _default_table_path), so a serving process does not stall its first
  requests on tuning every prefill / decode bucket again on a machine that has served before."""

  def __init__(self):
    self.mode = os.environ.get("XOT_GEMM", "auto")
    self.seeded = False
    self.table: Dict[Tuple, object] = {}
    self.path = None
    self._path_resolved = False
    self.capturing = False

  def _load(self, path: str) -> None:
    try:
      with open(path) as f:
        for k, v in json.load(f).items():
          if k.startswith("_"):  # comments
            continue
          self.table.setdefault(tuple(json.loads(k)), tuple(v) if isinstance(v, list) else v)
    except (OSError, ValueError):
      pass  # a corrupt or unreadable table is only a cache

  def _table_path(self):
    """Resolved lazily (needs the device): loads the persisted table the first time a choice is needed, then the
    seed table under it (keys the box has not tuned itself)."""
    if not self._path_resolved:
      self._path_resolved = True
      self.path = _default_table_path()
      if self.path and os.path.exists(self.path):
        self._load(self.path)
      seed = _seed_table_path()
      if seed:
        self._load(seed)
        self.seeded = True
    return self.path

  def _lookup(self, key):
    self._table_path()
    return self.table.get(key)

  def _store(self, key, got):
    self.table[key] = got
    path = self._table_path()
    if path:
      try:
        self.dump(path)
      except OSError:
        pass

  def dump(self, path: str):
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    tmp = f"{path}.{os.getpid()}.tmp"
    with open(tmp, "w") as f:
      json.dump({json.dumps(list(k)): v for k, v in self.table.items()}, f, indent=1)
    os.replace(tmp, path)  # atomic: concurrent processes never read a half-written table

  _flush_buf = None

  @classmethod
  def _time(cls, fn) -> float:
    """Cold-cache time of one call: a 512 MB write before each rep evicts the weight from L2 and the
    256 MB MALL, as in a real forward pass where each layer's weights are read once per step."""
    if cls._flush_buf is None:
      cls._flush_buf = torch.empty(128 << 20, dtype=torch.float32, device=torch.cuda.current_device())
    fn()
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    times = []
    for _ in range(5):
      cls._flush_buf.fill_(0.0)
      st.record()
      fn()
      en.record()
      en.synchronize()
      times.append(st.elapsed_time(en))
    times.sort()
    return times[1]

  def stream8_cfg(self, x, w, bias, residual, epi, out_dtype) -> Tuple:
    """(ntw, split-K) of the FP8-weight stream GEMM at this M bucket (cold-cache timed once)."""
    M, Kd = x.shape
    N = w.shape[0]
    key = ("s8", _m_bucket(M), N, Kd, epi, bias is not None, str(out_dtype))
    got = self._lookup(key)
    if got is not None:
      return got
    cands = self._stream_cands(M, N, Kd, epi)
    if not cands:
      raise RuntimeError(f"no FP8 stream GEMM configuration for N={N} K={Kd}")
    if self._no_tuning():
      return self._heuristic(M, N, [("stream",) + c for c in cands])[1:]
    scratch.splitk(x.device, max(c[1] * M * N for c in cands))
    y = torch.empty(M, N // 2 if epi == "silu" else N, dtype=out_dtype, device=x.device)
    times = {}
    for cfg in cands:
      try:
        times[cfg] = self._time(lambda: _stream8_call(x, w, bias, residual, epi, y, cfg))
      except RuntimeError:
        pass
    got = min(times, key=times.get) if times else cands[0]
    self._store(key, got)
    return got

  def _no_tuning(self) -> bool:
    return self.capturing or torch.cuda.is_current_stream_capturing()

  # ---------------------------------------------------------------- row-major weights
  def choose(self, x, w, bias, residual, epi, out_dtype):
    """Row-major weight: the library's skinny/tiled GEMM ("hip") or the stream GEMM on the row-major layout
    (("stream", ntw, S)); cold-cache timed once per M bucket.  hipBLASLt ("blas") only when asked for
    (XOT_GEMM=blas, or XOT_GEMM_BLAS=1 to time it among the candidates) -- every weight the models run hot is
    pre-shuffled, so row-major weights are the odd shapes that layout does not tile."""
    if self.mode in ("hip", "blas"):
      return self.mode
    M, Kd = x.shape
    N = w.shape[0]
    key = ("rm", _m_bucket(M), N, Kd, epi, bias is not None)
    got = self._lookup(key)
    if got is not None:
      return got
    if self._no_tuning():
      return "hip"
    cands = ["hip", "blas"] if BLAS_CAND else ["hip"]
    if M <= 256:
      cands += [("stream",) + c for c in self._stream_cands(M, N, Kd, epi)]
      scratch.splitk(x.device, 8 * max(M, 128) * N)
    times = {}
    res_copy = residual.clone() if residual is not None else None
    for impl in cands:
      try:
        times[impl] = self._time(lambda: _run_rowmajor(impl, x, w, bias, res_copy, epi, None, out_dtype))
      except RuntimeError:
        times[impl] = float("inf")
    got = min(times, key=times.get)
    if times[got] == float("inf"):  # a shape none of the library's kernels tiles (e.g. a 300-row LM head)
      got = "blas"
    self._store(key, got)
    return got

  @staticmethod
  def _stream_cands(M, N, Kd, epi):
    cands = []
    for ntw in ((2, 4) if epi == "silu" else (1, 2, 4)):
      if N % (64 * ntw) or (ntw == 4 and M <= 32):
        continue
      for S in (1, 2, 4, 8):
        if Kd % (S * 128) == 0 and (N // (64 * ntw)) * S <= 4096:
          cands.append((ntw, S))
    return cands

  # ---------------------------------------------------------------- shuffled weights
  @staticmethod
  def _big_cands(M, N, Kd):
    cands = []
    if N % 16:
      return cands
    # 1256 / 2256: the 256 x 256 tile on the two-group ping-pong schedule in four / two phases per stage
    codes = [256, 1256, 2256, 128] if PP2 else [256, 1256, 128]
    if W4 and N % 256 == 0:  # four-wave 256 x 256 tile (csrc/gemm_w4.hip): 256-row tiles only
      codes.append(4256)
    if N % 224 == 0:  # 7 row groups per wave: whole rounds where 256-wide tiles leave a half round (8B gate/up)
      codes.append(224)
    bm = big_row_tile(M)
    if bm < 256:  # rows that would leave >= 32 padding rows in 256-row tiles: shorter row tiles (two-phase: 192 only)
      codes += [bm * 10000 + 256, bm * 10000 + 128] + ([bm * 10000 + 2256] if PP2 and bm == 192 else [])
    for bn in codes:
      if N % tile_width(bn) and N < tile_width(bn):  # a partial last column tile is masked; skip tiles wider than N
        continue
      tiles = -(-M // tile_rows(bn)) * -(-N // tile_width(bn))
      for S in (1, 2, 3, 4, 6, 8):
        if S > 1 and (tiles >= 256 or tiles * S > 1024 or Kd // 64 < 2 * S):
          continue
        cands.append(("big", bn, S))
    return cands

  def shuffled_cfg(self, x, w, bias, residual, epi, out_dtype) -> Tuple:
    """(kernel, ntw | bn, split-K) for a pre-shuffled weight at this M bucket."""
    M, Kd = x.shape
    N = w.shape[0]
    key = ("sh", _m_bucket(M), N, Kd, epi, bias is not None, str(out_dtype))
    got = self._lookup(key)
    if got is not None:
      return got
    if (TALL_FIXED and W4 and M >= W4_PREF_M and N % 256 == 0 and Kd % 128 == 0
        and not (epi == "resid" and out_dtype == torch.float32) and M * x.stride(0) * 2 < (1 << 32)):
      # (the last term: the tile's LDS-DMA loads take 32-bit byte offsets into X; taller / wider X take the
      # tuned candidates below)
      # tall GEMMs (prefill chunks, training): the four-wave tile at S = 1 won every tuned tall shape this round
      # (profiles/r5/headline/bench_r5o_tunelog.log), so it is taken without the cold-timing pass, which cost
      # ~0.5 s inside the first prefill chunk of every fresh process
      got = ("big", 4256, 1)
      self._store(key, got)
      return got
    cands = []
    if M <= STREAM_MAX_M:
      cands += [("stream",) + c for c in self._stream_cands(M, N, Kd, epi)]
    if M >= BIG_MIN_M and Kd % 128 == 0:
      cands += self._big_cands(M, N, Kd)
    if not cands:
      raise RuntimeError(f"no GEMM configuration for pre-shuffled N={N} K={Kd} M={M}")
    if self._no_tuning():
      return self._heuristic(M, N, cands)
    scratch.splitk(x.device, max(_ws_elems(c, M, N) for c in cands))
    y = torch.empty(M, N // 2 if epi == "silu" else N, dtype=out_dtype, device=x.device)
    times = {}
    for cfg in cands:
      try:
        times[cfg] = self._time(lambda: _shuffled_call(x, w, bias, residual, epi, y, cfg)) + _slab_read_ms(cfg, M, N)
      except RuntimeError:
        pass
    got = _tie_break(times, M) if times else cands[0]
    if TUNE_LOG:
      print(f"[gemm tune] {key} -> {got}: " + ", ".join(f"{c}={t * 1e3:.1f}us" for c, t in sorted(times.items(), key=lambda i: i[1])),
            file=sys.stderr, flush=True)
    self._store(key, got)
    return got

  @staticmethod
  def _heuristic(M, N, cands):
    if not any(c[0] in ("big", "stream") for c in cands):
      return cands[0]
    if M <= 128 or not any(c[0] == "big" for c in cands):
      best = None  # stream GEMM: enough workgroups to cover 256 CUs a few times
      for c in cands:
        if c[0] != "stream":
          continue
        wg = (N // (64 * c[1])) * c[2]
        score = abs(wg - 768)
        if best is None or score < best[0]:
          best = (score, c)
      return best[1]
    best = None  # big GEMM: split K until the tiles cover the CUs once
    for c in cands:
      if c[0] != "big":
        continue
      tiles = -(-M // tile_rows(c[1])) * (N // tile_width(c[1])) * c[2]
      score = abs(tiles - 256) + (0 if c[1] == (2256 if PP2 else 1256) else 64)
      if best is None or score < best[0]:
        best = (score, c)
    return best[1]


# Isolated timings of 256-row tile variants at the same K split land within a few percent of each other and the
# winner changes from run to run, but inside a whole decode step (back to back, at the power cap) the ping-pong
# 256 x 256 tile (two-phase first) is the measured winner (a 256 x 224 gate/up or plain-256 qkv pick cost ~2 % of the headline step,
# profiles/r4/tuner/slab_penalty/, tie/: a plain-256 down pick 82.49 vs 81.91 / 81.83 ms): within TIE of the
# fastest, prefer it.
TIE = float(os.environ.get("XOT_GEMM_TIE", "0.05"))
# ... and across K splits, the two-phase tile within TIE_X of the fastest: the isolated timing runs below the power
# cap, where a sparser MFMA schedule gains most from the higher clock.  Llama-3-70B o-proj at 512 rows: timed
# 256 x 128 S 2 84.3 us vs two-phase S 4 92.7 us, but in the step the two-phase pick is 0.5 ms faster (78.30 vs
# 78.82 / 78.86 ms, profiles/r4/tuner/oproj/)
TIE_X = float(os.environ.get("XOT_GEMM_TIE_X", "0.10"))
TUNE_LOG = os.environ.get("XOT_GEMM_TUNE_LOG", "0") == "1"  # print every shuffled-weight tuning's timings
_BIG_PREF = {2256: 0, 4256: 1, 1256: 2, 256: 3, 224: 4, 128: 5}
_BIG_PREF_TALL = {4256: 0, 2256: 1, 1256: 2, 256: 3, 224: 4, 128: 5}


def _tie_break(times: Dict, M: int = 0) -> Tuple:
  best = min(times, key=times.get)
  code = lambda c: c[1] % 10000  # noqa: E731 - the schedule, whatever the row tile
  if best[0] != "big" or code(best) not in _BIG_PREF or TIE <= 0:
    return best
  pref = _BIG_PREF_TALL if M >= W4_PREF_M else _BIG_PREF
  top = min(pref, key=pref.get)
  close = [c for c, t in times.items()
           if c[0] == "big" and code(c) in pref and ((c[2] == best[2] and t <= times[best] * (1 + TIE))
                                                     or (code(c) == top and t <= times[best] * (1 + TIE_X)))]
  return min(close, key=lambda c: (pref[code(c)], times[c]))


def _ws_elems(cfg, M, N) -> int:
  return cfg[2] * M * N if len(cfg) == 3 and cfg[2] > 1 else 0


# HBM rate (TB/s) at which the consumer of split-K fp32 slabs (slab reduce, fused reduce + RoPE / + residual +
# RMSNorm) reads them back: a K-split candidate's timed GEMM is charged that read, so the tuner ranks the
# GEMM + reduce pair rather than the GEMM alone (XOT_SLAB_TBPS=0: GEMM time only)
SLAB_TBPS = float(os.environ.get("XOT_SLAB_TBPS", "5.0"))


def _slab_read_ms(cfg, M, N) -> float:
  n = _ws_elems(cfg, M, N)
  return n * 4 / (SLAB_TBPS * 1e9) if n and SLAB_TBPS > 0 else 0.0


policy = GemmPolicy()


def _stream_call(x, w, bias, residual, epi, out, cfg, shuffled: bool = True):
  ntw, S = cfg
  M, N = x.shape[0], w.shape[0]
  ws = scratch.splitk(x.device, S * M * N) if S > 1 else None
  require().gemm_stream(x, w, out, bias, residual, ws, K.EPI[epi], ntw, S, shuffled)
  return out


def _stream8_call(x, w, bias, residual, epi, out, cfg):
  ntw, S = cfg
  M, N = x.shape[0], w.shape[0]
  ws = scratch.splitk(x.device, S * M * N) if S > 1 else None
  require().gemm_stream8(x, w, w.xot_scale, out, bias, residual, ws, K.EPI[epi], ntw, S)
  return out


# FP8 weights: largest M for the FP8 stream GEMM; above it the weight is widened to a bf16 scratch copy
STREAM8_MAX_M = int(os.environ.get("XOT_STREAM8_MAX_M", "256"))


def _linear8(x, w, bias, residual, epi, out, dt):
  M, N = x.shape[0], w.shape[0]
  if M > STREAM8_MAX_M:  # compute-bound: widen once per call (straight into the bf16 tile layout), then gemm_big
    wb = dequant_stream8_to_stream(w, w.xot_scale)
    wb.xot_layout = "stream"
    return linear(x, wb, bias=bias, residual=residual, epi=epi, out=out, out_dtype=dt)
  if out is None:
    out = torch.empty(M, N // 2 if epi == "silu" else N, dtype=dt, device=x.device)
  if x.stride(1) != 1 or x.stride(0) % 8:
    x = x.contiguous()
  return _stream8_call(x, w, bias, residual, epi, out, policy.stream8_cfg(x, w, bias, residual, epi, dt))


def _shuffled_call(x, w, bias, residual, epi, out, cfg):
  if cfg[0] == "stream":
    return _stream_call(x, w, bias, residual, epi, out, cfg[1:])
  _, bn, S = cfg
  M, N = x.shape[0], w.shape[0]
  ws = scratch.splitk(x.device, S * M * N) if S > 1 else None
  require().gemm_big(x, w, out, bias, residual, ws, K.EPI[epi], bn, S)
  return out


def _run_rowmajor(impl, x, w, bias, residual, epi, out, out_dtype):
  if impl == "hip":
    return K.gemm(x, w, bias=bias, residual=residual, epi=epi, out=out, out_dtype=out_dtype)
  if isinstance(impl, tuple) and impl[0] == "stream":
    M, N = x.shape[0], w.shape[0]
    if out is None:
      out = torch.empty(M, N // 2 if epi == "silu" else N, dtype=out_dtype or x.dtype, device=x.device)
    return _stream_call(x.contiguous(), w, bias, residual, epi, out, impl[1:], shuffled=False)
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


# XOT_FUSE_NORM=0: batch-1 decode keeps the separate split-K reduce + residual + RMSNorm launch after o_proj /
# down_proj (fused: the next GEMM recomputes the norm of the pending slabs in its prologue, csrc/gemm.hip NORM)
FUSE_NORM = os.environ.get("XOT_FUSE_NORM", "1") != "0"
# XOT_FUSE_MERGE=0: batch-1 decode keeps the attention's partition-merge launch (fused: o_proj merges the partitions
# of its K slice in its prologue, csrc/gemm.hip MERGE; only together with the deferred norm above)
FUSE_MERGE = os.environ.get("XOT_FUSE_MERGE", "1") != "0"
# widest residual row whose norm is deferred: every consumer workgroup re-reads the row and all its slabs, which paid
# at 4096 (Llama-3-8B 3.50 -> 3.33 ms/token) but not at 8192 (Llama-3-70B 23.97 vs 24.07 ms, profiles/r6/headline/b1/)
DEFER_MAX_D = 4096


class PendingNorm:
  """rmsnorm(bf16(src + bias + sum of the S fp32 slabs in ws)) * ln_w, not computed yet.

  A residual projection of a batch-1 decode step (linear_resid_norm with defer_to) leaves its split-K slabs; the
  next GEMM (linear with epi none / silu, linear_rope_kv) folds the slab sum, the residual add and the RMSNorm into
  its prologue (gemm_stream_norm) and stores the summed residual row into dst -- a buffer distinct from src, since
  every workgroup of that GEMM reads src.  Any other consumer calls materialize(), the unfused kernel, which
  leaves the same residual in dst.  After either, dst is the residual stream."""

  __slots__ = ("src", "dst", "ws", "S", "bias", "ln_w", "eps")

  def __init__(self, src, dst, ws, S, bias, ln_w, eps):
    self.src, self.dst, self.ws, self.S, self.bias, self.ln_w, self.eps = src, dst, ws, S, bias, ln_w, float(eps)

  @property
  def shape(self):
    return self.src.shape

  def materialize(self) -> torch.Tensor:
    if self.dst.data_ptr() != self.src.data_ptr():
      self.dst.copy_(self.src)
    out = torch.empty_like(self.dst)
    require().splitk_resid_rmsnorm(self.ws, self.S, self.bias, self.dst, self.ln_w, out, self.eps)
    return out

  def run(self, w: torch.Tensor, y: torch.Tensor, bias, epi: str, ntw: int, S: int, reduce: bool) -> None:
    ws = scratch.splitk(y.device, S * w.shape[0]) if S > 1 else None
    require().gemm_stream_norm(w, y, bias, ws, K.EPI[epi], ntw, S, reduce, self.src, self.ws, self.S, self.bias,
                               self.ln_w, self.dst, self.eps)


def _pending_cfg(p: PendingNorm, w: torch.Tensor, bias, epi: str):
  """The stream configuration the consumer GEMM of a pending norm runs (tuned on the unfused kernel with the
  residual row as a stand-in input), or None when the fused kernel does not cover it."""
  if layout_of(w) != "stream" or epi not in ("none", "silu") or w.shape[1] != p.src.shape[1]:
    return None
  cfg = policy.shuffled_cfg(p.src, w, bias, None, epi, torch.bfloat16)
  if cfg[0] != "stream" or w.shape[1] % (cfg[2] * 128) or (w.shape[1] // cfg[2]) * 2 > 65536:
    return None
  return cfg


def linear(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor | None = None, residual: torch.Tensor | None = None,
           epi: str = "none", out: torch.Tensor | None = None, out_dtype: torch.dtype | None = None) -> torch.Tensor:
  if isinstance(x, PendingNorm):
    cfg = None if (residual is not None or (out_dtype not in (None, torch.bfloat16))
                   or (out is not None and out.dtype != torch.bfloat16)) else _pending_cfg(x, w, bias, epi)
    if cfg is None:
      x = x.materialize()
    else:
      if out is None:
        out = torch.empty(1, w.shape[0] // 2 if epi == "silu" else w.shape[0], dtype=torch.bfloat16,
                          device=x.src.device)
      x.run(w, out, bias, epi, cfg[1], cfg[2], True)
      return out
  if not x.is_cuda:
    return K.gemm(x, to_rowmajor(w), bias=bias, residual=residual, epi=epi, out=out, out_dtype=out_dtype)
  dt = out_dtype or (out.dtype if out is not None else x.dtype)
  M, N = x.shape[0], w.shape[0]
  if layout_of(w) == "stream8":
    return _linear8(x, w, bias, residual, epi, out, dt)
  if layout_of(w) != "stream":
    impl = policy.choose(x, w, bias, residual, epi, dt)
    return _run_rowmajor(impl, x, w, bias, residual, epi, out, out_dtype)
  if out is None:
    out = torch.empty(M, N // 2 if epi == "silu" else N, dtype=dt, device=x.device)
  if x.stride(1) != 1 or x.stride(0) % 8:
    x = x.contiguous()
  cfg = policy.shuffled_cfg(x, w, bias, residual, epi, dt)
  _shuffled_call(x, w, bias, residual, epi, out, cfg)
  return out




def linear_resid_norm(x: torch.Tensor, w: torch.Tensor, h: torch.Tensor, ln_w: torch.Tensor, eps: float,
                      bias: torch.Tensor | None = None, out: torch.Tensor | None = None,
                      defer_to: torch.Tensor | None = None):
  """h += x @ w.T (+ bias) in place (the residual stream) and return rmsnorm(h) * ln_w.

  When the projection runs split-K on the pre-shuffled layout, the GEMM leaves its fp32 slabs and one
  kernel does the slab reduce, the residual add and the RMSNorm (instead of reduce + norm kernels).
  defer_to (a second residual buffer, one row): return a PendingNorm instead -- the slabs stay for the next
  GEMM's prologue, and the residual stream continues in defer_to (h is left as it was).
  x may be a kernels.PendingMerge (batch-1 decode attention): with defer_to, the projection merges the attention's
  partitions in its own prologue (gemm_stream_merge); otherwise the merge kernel runs first."""
  if isinstance(x, K.PendingMerge):
    xm = x.out.view(x.out.shape[0], -1)  # [1, H * Dh]; the stand-in operand of the configuration choice
    if defer_to is not None and FUSE_NORM and layout_of(w) == "stream" and xm.shape[0] == 1:
      N, Kd = w.shape
      cfg = policy.shuffled_cfg(xm, w, bias, h, "resid", h.dtype)
      if (cfg[0] == "stream" and 1 < cfg[2] <= 8 and Kd % (cfg[2] * 128) == 0 and (Kd // cfg[2]) * 2 <= 65536
          and h.is_contiguous() and h.dtype == torch.bfloat16):
        S = cfg[2]
        if N <= DEFER_MAX_D and out is None:  # merge here, norm in the next GEMM's prologue
          ws = scratch.splitk(h.device, S * N, slot=1)
          require().gemm_stream_merge(w, ws, cfg[1], S, x.o, x.ml, x.ctx_lens, x.ppp, x.nparts, x.out.shape[-1])
          return PendingNorm(h, defer_to, ws, S, bias, ln_w, eps)
        ws = scratch.splitk(h.device, S * N)  # merge here, then the usual slab reduce + residual + norm
        require().gemm_stream_merge(w, ws, cfg[1], S, x.o, x.ml, x.ctx_lens, x.ppp, x.nparts, x.out.shape[-1])
        out = torch.empty_like(h) if out is None else out
        require().splitk_resid_rmsnorm(ws, S, bias, h, ln_w, out, float(eps))
        return out
    x = x.materialize().view(xm.shape)
  if x.is_cuda and layout_of(w) == "stream":
    if x.stride(1) != 1 or x.stride(0) % 8:
      x = x.contiguous()
    M, N = x.shape[0], w.shape[0]
    cfg = policy.shuffled_cfg(x, w, bias, h, "resid", h.dtype)
    if (defer_to is not None and FUSE_NORM and M == 1 and cfg[0] == "stream" and 1 < cfg[2] <= 8 and N <= DEFER_MAX_D
        and out is None and h.is_contiguous() and h.dtype == torch.bfloat16):
      S = cfg[2]
      ws = scratch.splitk(x.device, S * M * N, slot=1)
      require().gemm_stream(x, w, h, None, h, ws, K.EPI["resid"], cfg[1], S, True, False)
      return PendingNorm(h, defer_to, ws, S, bias, ln_w, eps)
    if cfg[0] in ("stream", "big") and cfg[2] > 1:
      S = cfg[2]
      ws = scratch.splitk(x.device, S * M * N)
      C = require()
      if cfg[0] == "stream":
        C.gemm_stream(x, w, h, None, h, ws, K.EPI["resid"], cfg[1], S, True, False)
      else:
        C.gemm_big(x, w, h, None, h, ws, K.EPI["resid"], cfg[1], S, False)
      out = torch.empty_like(h) if out is None else out
      C.splitk_resid_rmsnorm(ws, S, bias, h, ln_w, out, float(eps))
      return out
  linear(x, w, bias=bias, residual=h, epi="resid", out=h)
  return K.rmsnorm(h, ln_w, eps, out=out)[0]




def linear_rope_kv(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor | None, pos: torch.Tensor,
                   cos_sin: torch.Tensor, slots: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, H: int,
                   Hkv: int) -> torch.Tensor:
  """qkv = x @ w.T (+ bias); returns rope(q) [T, H, Dh] and writes rope(k), v into the paged caches.

  When the QKV projection runs split-K on the pre-shuffled layout, its fp32 slabs go straight to one
  kernel that sums them, rotates and writes q / the caches (no bf16 qkv round trip, one launch less).
  x may be a PendingNorm: the projection then computes its input row in its prologue."""
  if isinstance(x, PendingNorm):
    cfg = _pending_cfg(x, w, bias, "none")
    if cfg is None or cfg[2] < 2:
      x = x.materialize()
    else:
      S, N = cfg[2], w.shape[0]
      y = torch.empty(1, N, dtype=torch.bfloat16, device=x.src.device)  # shape carrier only
      x.run(w, y, None, "none", cfg[1], S, False)
      Dh = k_cache.shape[-1]
      q = torch.empty(1, H, Dh, dtype=torch.bfloat16, device=y.device)
      ws = scratch.splitk(y.device, S * N)
      require().splitk_rope_kv_write(ws, S, bias, pos, cos_sin, slots, q, k_cache, v_cache, int(H), int(Hkv))
      return q
  if x.is_cuda and layout_of(w) == "stream":
    if x.stride(1) != 1 or x.stride(0) % 8:
      x = x.contiguous()
    M, N = x.shape[0], w.shape[0]
    cfg = policy.shuffled_cfg(x, w, bias, None, "none", x.dtype)
    if cfg[0] in ("stream", "big") and cfg[2] > 1:
      S = cfg[2]
      ws = scratch.splitk(x.device, S * M * N)
      y = torch.empty(M, N, dtype=x.dtype, device=x.device)  # shape carrier only: the slabs are not reduced
      C = require()
      if cfg[0] == "stream":
        C.gemm_stream(x, w, y, None, None, ws, K.EPI["none"], cfg[1], S, True, False)
      else:
        C.gemm_big(x, w, y, None, None, ws, K.EPI["none"], cfg[1], S, False)
      Dh = k_cache.shape[-1]
      q = torch.empty(M, H, Dh, dtype=x.dtype, device=x.device)
      C.splitk_rope_kv_write(ws, S, bias, pos, cos_sin, slots, q, k_cache, v_cache, int(H), int(Hkv))
      return q
  qkv = linear(x, w, bias=bias)
  return K.rope_kv_write(qkv, pos, cos_sin, slots, k_cache, v_cache, H, Hkv)

"""Python entry points of the gfx950 kernel library.

Each function takes torch tensors, allocates outputs when the caller did not preallocate them, and
dispatches to the HIP kernel for GPU tensors or to the fp32 torch reference (`ops.reference`) for
CPU tensors.  GPU tensors never take the reference path: if the extension is missing the call
raises (see `ops._ext.require`).
"""
from __future__ import annotations

import os

import torch

from . import reference as ref
from ._ext import require

EPI = {"none": 0, "resid": 1, "silu": 2}
PAGE = 64


def _gpu(t: torch.Tensor) -> bool:
  if t.is_cuda:
    require()
    return True
  return False


# ------------------------------------------------------------------ norms / elementwise
def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float, residual: torch.Tensor | None = None,
            out: torch.Tensor | None = None, residual_out: torch.Tensor | None = None):
  """Returns (out, residual_out).  With `residual`, residual_out = x + residual (the new stream)."""
  if not _gpu(x):
    y, r = ref.rmsnorm(x, w, eps, residual)
    if out is not None:
      out.copy_(y)
      y = out
    if residual_out is not None and r is not None:
      residual_out.copy_(r)
      r = residual_out
    return y, r
  out = torch.empty_like(x) if out is None else out
  if residual is not None and residual_out is None:
    residual_out = torch.empty_like(x)
  require().rmsnorm(x, w, out, residual, residual_out, float(eps))
  return out, residual_out


def embedding(ids: torch.Tensor, table: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
  if not _gpu(table):
    y = table[ids.long().clamp(0, table.shape[0] - 1)]
    if out is not None:
      out.copy_(y.reshape(out.shape))
      return out
    return y
  ids32 = ids.to(torch.int32).contiguous()
  out = torch.empty(ids32.numel(), table.shape[1], dtype=table.dtype, device=table.device) if out is None else out
  require().embedding(ids32, table, out)
  return out


def silu_mul(gu: torch.Tensor, out: torch.Tensor | None = None, interleaved16: bool = False) -> torch.Tensor:
  """silu(gate) * up.  gu = [gate | up] halves, or 16-column interleaved tiles (fused gate_up layout)."""
  if not _gpu(gu):
    if interleaved16:
      M, N = gu.shape
      g = gu.view(M, N // 32, 2, 16)
      y = (torch.nn.functional.silu(g[:, :, 0].float()) * g[:, :, 1].float()).reshape(M, N // 2).to(gu.dtype)
    else:
      y = ref.silu_mul(gu)
    if out is not None:
      out.copy_(y)
      return out
    return y
  Fd = gu.shape[-1] // 2
  out = torch.empty(*gu.shape[:-1], Fd, dtype=gu.dtype, device=gu.device) if out is None else out
  require().silu_mul(gu.contiguous(), out, bool(interleaved16))
  return out


# ------------------------------------------------------------------ GEMM
def gemm(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor | None = None, residual: torch.Tensor | None = None,
         epi: str = "none", out: torch.Tensor | None = None, out_dtype: torch.dtype | None = None, algo: int = 0,
         nt: int = 0) -> torch.Tensor:
  """y = x @ w.T (+bias) with fused epilogue: 'none' | 'resid' (y += residual) | 'silu'.

  For 'silu' the weight rows must be gate/up interleaved in 16-row tiles (see
  models.weights.interleave_gate_up); the output has w.shape[0] // 2 columns.
  """
  M, N = x.shape[0], w.shape[0]
  ncol = N // 2 if epi == "silu" else N
  if not _gpu(x):
    y = ref.linear(x, w, bias)
    if epi == "silu":
      y = y.view(M, N // 32, 2, 16)
      y = (torch.nn.functional.silu(y[:, :, 0]) * y[:, :, 1]).reshape(M, ncol)
    elif epi == "resid":
      y = y + residual.float()
    dt = out_dtype or (out.dtype if out is not None else x.dtype)
    if out is not None:
      out.copy_(y.to(out.dtype))
      return out
    return y.to(dt)
  if out is None:
    out = torch.empty(M, ncol, dtype=out_dtype or x.dtype, device=x.device)
  if nt == 0:
    nt = 2 if (N // 32) >= 1024 else 1
  if algo == 0 and epi != "silu" and N % 16:  # the skinny kernel tiles 16 output columns; the tiled one masks
    algo = 2
  require().gemm(x, w, out, bias, residual, EPI[epi], int(algo), int(nt))
  return out


# ------------------------------------------------------------------ RoPE + paged KV
def rope_kv_write(qkv: torch.Tensor, pos: torch.Tensor, cos_sin: torch.Tensor, slots: torch.Tensor,
                  k_cache: torch.Tensor, v_cache: torch.Tensor, H: int, Hkv: int,
                  q_out: torch.Tensor | None = None) -> torch.Tensor:
  """qkv [T, (H+2Hkv)*Dh] -> rotated q [T, H, Dh]; rotated k and v written into the paged caches."""
  T = qkv.shape[0]
  Dh = k_cache.shape[-1]
  if not _gpu(qkv):
    x = qkv.view(T, H + 2 * Hkv, Dh)
    q = ref.rope(x[:, :H], pos, cos_sin)
    k = ref.rope(x[:, H:H + Hkv], pos, cos_sin)
    ref.write_kv(k, x[:, H + Hkv:], slots, k_cache, v_cache)
    if q_out is not None:
      q_out.copy_(q.view(q_out.shape))
      return q_out
    return q
  q_out = torch.empty(T, H, Dh, dtype=qkv.dtype, device=qkv.device) if q_out is None else q_out
  require().rope_kv_write(qkv, pos, cos_sin, slots, q_out, k_cache, v_cache, int(H), int(Hkv))
  return q_out


def rope_apply(x: torch.Tensor, pos: torch.Tensor, cos_sin: torch.Tensor, nh: int, Dh: int, inverse: bool = False,
               out: torch.Tensor | None = None) -> torch.Tensor:
  """x [T, >= nh*Dh] (2-D rows) -> rotated copy (or into `out`)."""
  if not _gpu(x):
    y = ref.rope(x[:, :nh * Dh].reshape(-1, nh, Dh), pos, cos_sin, inverse).reshape(x.shape[0], nh * Dh)
    if out is not None:
      out[:, :nh * Dh].copy_(y)
      return out
    return y
  out = torch.empty(x.shape[0], nh * Dh, dtype=x.dtype, device=x.device) if out is None else out
  require().rope_apply(x, out, pos, cos_sin, int(nh), int(Dh), bool(inverse))
  return out


# ------------------------------------------------------------------ attention
# 0: workgroup per (sequence, KV head, partition), waves split pages + LDS combine
# 1 / 2: wave per (sequence, KV head, partition), transposed S^T (lane = query head), no LDS;
#        2 prefetches the next page under the current one
# 3: 2 with non-temporal K / V loads (neutral in round 3, profiles/r3/s3/; on the chunk-major V cache of round 6
#        the KV stream runs 5-13 % faster in isolation -- B 512: 183.9 vs 193.7 us per layer, B 256 / ctx 1040:
#        166.6 vs 185.1, B 128 / ctx 2048: 156.2 vs 177.3 -- and the 70B headline step 74.6-74.7 vs 75.4-75.7 ms,
#        profiles/r6/headline/attn_nt/)
# -1 (default): 0 below 64 (sequence, KV head) pairs -- few long sequences, where the workgroup
#        kernel's 4-wave page split needs fewer partitions; else 3 once a layer's K / V pages (batch x block-table
#        width) outgrow the 256 MB last-level cache, 2 below (B 16 / ctx 530: 15.1 vs 13.5 us, B 64 / ctx 530: 29.3 vs
#        24.8 with nt; B 16 / ctx 8192: 85.7 vs 97.1, B 64 / ctx 2048: 85.1 vs 97.2; tools/bench_attn_small.py,
#        profiles/r6/headline/attn_nt/attn_small.log)
# (4, an 8-wave workgroup over one partition for short tables at small batch, measured 1 % slower at 8B batch 1 --
#  3.55 vs 3.52 ms, profiles/r3/s3/ -- and was removed in round 6)
DECODE_ALGO = int(os.environ.get("XOT_ATTN_DECODE", "-1"))


NT_MIN_KV_BYTES = 256 << 20  # K / V bytes per layer from which the page loads go non-temporal (algo 3)


def resolve_decode_algo(batch: int, Hkv: int, algo: int | None = None, kv_bytes: int | None = None) -> int:
  algo = DECODE_ALGO if algo is None else algo
  if algo < 0:
    if batch * Hkv < 64:
      return 0
    return 3 if kv_bytes is None or kv_bytes >= NT_MIN_KV_BYTES else 2
  return algo


def choose_pages_per_part(batch: int, Hkv: int, max_ctx: int, algo: int | None = None) -> int:
  """KV pages per split-KV partition for a decode step of `batch` sequences."""
  algo = resolve_decode_algo(batch, Hkv, algo)
  pages = max(1, -(-max_ctx // PAGE))
  if algo == 0:  # enough workgroups to cover 256 CUs several times, >= 4 pages (one per wave) each
    for ppp in (16, 8, 4):
      if batch * Hkv * -(-pages // ppp) >= 1024:
        return ppp
    return 4
  # one wave per unit: ~1024 waves (4 per CU), partitions of 2..32 pages (tools/bench_attn_small.py,
  # profiles/bench_attn_small_r1.json: 2048 waves of shorter partitions lose to the extra merge work)
  nparts = max(1, min(max(pages // 2, 1), -(-1024 // max(batch * Hkv, 1))))
  nparts = max(nparts, -(-pages // 32))
  return -(-pages // nparts)


class DecodeWorkspace:
  """Split-KV scratch for attn_decode, sized for every batch up to max_batch at this context bound.
  The partitioning is chosen per call from the actual batch (static per captured graph)."""

  def __init__(self, max_batch: int, H: int, Dh: int, max_ctx: int, device, pages_per_part: int | None = None,
               algo: int | None = None):
    self.algo = DECODE_ALGO if algo is None else algo
    self.max_ctx = max_ctx
    self.Hkv_hint = None
    self.Dh = Dh
    self.fixed_ppp = pages_per_part
    pages = max(1, -(-max_ctx // PAGE))
    worst = 1
    for b in range(1, max_batch + 1):
      for hkv in (1, 2, 4, 8, 16):
        ppp = pages_per_part or choose_pages_per_part(b, hkv, max_ctx, self.algo)
        worst = max(worst, b * -(-pages // ppp))
    self.units = worst  # max over batch of batch * nparts
    self.o = torch.empty(worst * H * Dh, dtype=torch.float32, device=device)
    self.ml = torch.empty(worst * H * 2, dtype=torch.float32, device=device)

  def partition(self, batch: int, Hkv: int, width_pages: int):
    """(pages per partition, partitions, kernel) for this call."""
    algo = resolve_decode_algo(batch, Hkv, self.algo, kv_bytes=batch * Hkv * width_pages * PAGE * self.Dh * 4)
    ppp = self.fixed_ppp or choose_pages_per_part(batch, Hkv, width_pages * PAGE, algo)
    nparts = max(1, -(-width_pages // ppp))
    if batch * nparts > self.units:
      raise RuntimeError(f"decode workspace sized for {self.units} units, need {batch * nparts}")
    return ppp, nparts, algo


class PendingMerge:
  """A batch-1 split-KV decode attention whose partition merge was left to its consumer: o_proj merges the
  partitions of its K slice in its GEMM prologue (linear_resid_norm -> gemm_stream_merge), one launch less per
  layer.  materialize() runs the merge kernel into `out` instead."""

  __slots__ = ("o", "ml", "ctx_lens", "ppp", "nparts", "out")

  def __init__(self, o, ml, ctx_lens, ppp, nparts, out):
    self.o, self.ml, self.ctx_lens, self.ppp, self.nparts, self.out = o, ml, ctx_lens, ppp, nparts, out

  def materialize(self) -> torch.Tensor:
    require().attn_decode_merge(self.o, self.ml, self.ctx_lens, self.out, self.ppp, self.nparts)
    return self.out


def attn_decode(q, k_cache, v_cache, block_tables, ctx_lens, scale: float, ws: DecodeWorkspace | None = None,
                out: torch.Tensor | None = None, defer_merge: bool = False):
  """defer_merge (one sequence): return a PendingMerge when the context is split over partitions."""
  if not _gpu(q):
    y = ref.attn_decode(q, k_cache, v_cache, block_tables, ctx_lens, scale)
    if out is not None:
      out.copy_(y.view(out.shape))
      return out
    return y
  B, H, Dh = q.shape
  width = block_tables.shape[1]
  if ws is None:
    ws = DecodeWorkspace(B, H, Dh, width * PAGE, q.device)
  ppp, nparts, algo = ws.partition(B, k_cache.shape[1], width)
  out = torch.empty_like(q) if out is None else out
  defer = defer_merge and B == 1 and nparts > 1
  require().attn_decode(q, k_cache, v_cache, block_tables, ctx_lens, out, ws.o, ws.ml, ppp, nparts, float(scale),
                        algo, not defer)
  return PendingMerge(ws.o, ws.ml, ctx_lens, ppp, nparts, out) if defer else out


# XOT_PREFILL_ATTN: 2 = 256-row workgroups, LDS-DMA page ring, in-register softmax (default); 1 = the
# first 64-row kernel (register-staged pages, P through LDS)
PREFILL_ALGO = int(os.environ.get("XOT_PREFILL_ATTN", "2"))


def attn_prefill(q, k_cache, v_cache, block_tables, cu_q, ctx_lens, max_qlen: int, scale: float,
                 out: torch.Tensor | None = None) -> torch.Tensor:
  if not _gpu(q):
    y = ref.attn_prefill(q, k_cache, v_cache, block_tables, cu_q, ctx_lens, scale)
    if out is not None:
      out.copy_(y)
      return out
    return y
  out = torch.empty_like(q) if out is None else out
  require().attn_prefill(q, k_cache, v_cache, block_tables, cu_q, ctx_lens, out, int(max_qlen), float(scale),
                         PREFILL_ALGO)
  return out


# ------------------------------------------------------------------ sampling
def attention_bidir(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, B: int, L: int, H: int, Dh: int,
                    scale: float) -> torch.Tensor:
  """Bidirectional (unmasked) multi-head attention over B sequences of L tokens: q / k / v [B*L, H*Dh] token-major
  (row views with unit inner stride) -> o [B*L, H*Dh].  GPU: the flash-style forward of the training kernels with
  the causal mask off (csrc/attention_train.hip; V transposed per head first) for Dh 64 / 128; CPU and other
  head sizes (the tiny test towers): fp32 reference."""
  if not _gpu(q) or Dh not in (64, 128):
    qh, kh, vh = (t.float().reshape(B, L, H, Dh).transpose(1, 2) for t in (q, k, v))
    a = torch.softmax((qh @ kh.transpose(-1, -2)) * scale, -1) @ vh
    return a.transpose(1, 2).reshape(B * L, H * Dh).to(q.dtype)
  C = require()
  Lp = -(-L // 64) * 64
  vt = torch.empty(B, H, Dh, Lp, dtype=v.dtype, device=v.device)
  C.attn_train_transpose(v, vt, B, L, Lp, H, Dh)
  o = torch.empty(B * L, H * Dh, dtype=q.dtype, device=q.device)
  lse2 = torch.empty(B * H * L, dtype=torch.float32, device=q.device)
  C.attn_train_fwd(q, k, vt, o, lse2, B, L, Lp, H, H, Dh, float(scale), False)
  return o


def sample(logits: torch.Tensor, temps: torch.Tensor, top_k: int, seed_off: torch.Tensor,
           out: torch.Tensor | None = None) -> torch.Tensor:
  """Greedy when temp <= 1e-5, else top-k + exponential-race sampling (all on device)."""
  if not _gpu(logits):
    B = logits.shape[0]
    res = torch.empty(B, dtype=torch.int32)
    g = torch.Generator().manual_seed(int(seed_off[0]) * 1000003 + int(seed_off[1]))
    for b in range(B):
      t = float(temps[b])
      row = logits[b].float()
      if t <= 1e-5 or top_k == 1:
        res[b] = int(row.argmax())
        continue
      row = row / max(t, 1e-5)
      if 0 < top_k < row.numel():
        kth = torch.topk(row, top_k).values[-1]
        row = row.masked_fill(row < kth, float("-inf"))
      probs = torch.softmax(row, -1)
      q = torch.empty_like(probs).exponential_(1, generator=g)
      res[b] = int((probs / q).argmax())
    if out is not None:
      out.copy_(res)
      return out
    return res
  out = torch.empty(logits.shape[0], dtype=torch.int32, device=logits.device) if out is None else out
  require().sample(logits, temps, int(top_k), seed_off, out)
  return out


def topk_cand(logits: torch.Tensor, top_k: int, kc: int = 64) -> tuple:
  """Each row's top_k (value, index) candidates in [B, kc] buffers (unused slots -inf / -1): one vocab
  slice's contribution to a sampler that runs on another stage."""
  B = logits.shape[0]
  if not _gpu(logits):
    v, i = torch.topk(logits.float(), top_k, dim=-1)
    vals = torch.full((B, kc), float("-inf"))
    idx = torch.full((B, kc), -1, dtype=torch.int32)
    vals[:, :top_k] = v
    idx[:, :top_k] = i.int()
    return vals, idx
  vals = torch.empty(B, kc, dtype=torch.float32, device=logits.device)
  idx = torch.empty(B, kc, dtype=torch.int32, device=logits.device)
  require().topk_cand(logits, int(top_k), vals, idx)
  return vals, idx


# ------------------------------------------------------------------ DeepSeek MLA
def mla_prep(ckv, kv_ln, q, qpe_off: int, H: int, pos, cos_sin, slots, cache, eps: float) -> None:
  """ckv [T, >= DL+DR] (rows may be strided), q [T, ldq]: latent norm + rope + cache write, q_pe rotated
  in place."""
  if not _gpu(ckv):
    ref.mla_prep(ckv, kv_ln, q, qpe_off, H, pos, cos_sin, slots, cache, eps)
    return
  require().mla_prep(ckv, kv_ln, q, int(qpe_off), int(H), pos, cos_sin, slots, cache, float(eps))


class MLAWorkspace:
  """Split-KV scratch of the MLA attention kernel."""

  def __init__(self, max_tokens: int, H: int, DL: int, max_ctx: int, device):
    self.max_tokens, self.H, self.DL = max_tokens, H, DL
    self.pages = max(1, -(-max_ctx // PAGE))
    self.max_parts = max(self.partition(1, self.pages)[1], self.partition(8, self.pages)[1])
    units = max(max_tokens * self.max_parts, 1)
    self.o = torch.empty(units * H * DL, dtype=torch.float32, device=device)
    self.ml = torch.empty(units * H * 2, dtype=torch.float32, device=device)

  def wide(self, T: int) -> bool:
    """Many-head kernel (one workgroup covers up to 128 heads, each page loaded once for all of them) for
    >= 64 heads at batch sizes that fill the chip; the narrow kernel (a workgroup per 16 heads) keeps more
    workgroups in flight for a handful of tokens.  XOT_MLA_WIDE=0/1 forces either."""
    force = os.environ.get("XOT_MLA_WIDE")
    if force in ("0", "1"):
      return force == "1"
    return self.H >= 64 and T >= 8

  def partition(self, T: int, width_pages: int):
    """(pages per partition, partitions, wide): enough workgroups for 256 CUs (one per CU: the kernels
    hold two 73 KB pages in LDS); narrow-kernel partitions of at least 2 pages."""
    nhb = -(-self.H // 16)
    wide = self.wide(T)
    units = T * -(-nhb // 8) if wide else T * nhb
    want = max(1, -(-256 // max(units, 1)))
    cap = width_pages if wide else (width_pages // 2 if width_pages >= 2 else 1)
    nparts = max(1, min(want, cap))
    ppp = -(-width_pages // nparts)
    return ppp, -(-width_pages // ppp), wide


def mla_attn(q_lat, q_pe, cache, block_tables, cu_q, ctx_lens, scale: float, ws: MLAWorkspace | None = None,
             out: torch.Tensor | None = None) -> torch.Tensor:
  """q_lat [H, T, DL], q_pe [T, >= H*DR] (row-major, strided rows ok) -> o_lat [H, T, DL]."""
  if not _gpu(q_lat):
    y = ref.mla_attn(q_lat, q_pe, cache, block_tables, cu_q, ctx_lens, scale)
    if out is not None:
      out.copy_(y)
      return out
    return y
  H, T, DL = q_lat.shape
  width = block_tables.shape[1]
  if ws is None:
    ws = MLAWorkspace(T, H, DL, width * PAGE, q_lat.device)
  ppp, nparts, wide = ws.partition(T, width)
  if T * nparts > ws.max_tokens * ws.max_parts:
    ppp, nparts = width, 1
  out = torch.empty_like(q_lat) if out is None else out
  require().mla_attn(q_lat, q_pe, cache, block_tables, cu_q, ctx_lens, out, ws.o, ws.ml, int(ppp), int(nparts),
                     float(scale), int(wide))
  return out


_ROUTE_CNT = {}


def _route_counters(device) -> torch.Tensor:
  """Per-device expert counters of moe_route_ds: zero between launches (the kernel resets them)."""
  key = str(device)
  if key not in _ROUTE_CNT:
    _ROUTE_CNT[key] = torch.zeros(256, dtype=torch.int32, device=device)
  return _ROUTE_CNT[key]


def moe_route_ds(logits, bias, k: int, n_group: int, topk_group: int, method: int, sigmoid: bool, norm: bool,
                 scale: float, outs: tuple | None = None):
  """DeepSeekMoE routing.  GPU: (topw, topi, slot_of, sorted_tok, off) device tensors (graph-capturable;
  launches on one stream reuse the per-device counters in order); CPU: (topw [T, k], topi [T, k])."""
  if not _gpu(logits):
    return ref.moe_route_ds(logits, bias, k, n_group, topk_group, method, sigmoid, norm, scale)
  T, E = logits.shape
  dev = logits.device
  if outs is None:
    outs = (torch.empty(T * k, dtype=torch.float32, device=dev), torch.empty(T * k, dtype=torch.int32, device=dev),
            torch.empty(T * k, dtype=torch.int32, device=dev), torch.empty(T * k, dtype=torch.int32, device=dev),
            torch.empty(E + 1, dtype=torch.int32, device=dev))
  require().moe_route_ds(logits.contiguous(), bias, int(k), int(n_group), int(topk_group), int(method), bool(sigmoid),
                         bool(norm), float(scale), _route_counters(dev), *outs)
  return outs

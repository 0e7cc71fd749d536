"""ShardRunner: one pipeline shard on one device — weights, paged KV pool, request bookkeeping,
step-input construction and HIP-graph replay of decode steps.

Requests are independent: each owns pages in the shard's KV pool (native C++ BlockManager), so any
number of sequences can be in flight on a shard and a ring stage can interleave micro-batches.
Decode steps of a given padded batch size are captured once into a HIP graph (torch.cuda.CUDAGraph
is hipGraph on ROCm) and replayed: one host launch per shard step instead of ~10 kernels per layer.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Sequence

import torch

from ..inference.shard import Shard
from ..models.config import ModelConfig
from ..models.transformer import KVCache, ShardModel, StepInputs
from ..models.weights import ShardWeights, prepare_for_decode, random_weights
from ..ops import linear as linear_mod

PAGE = 64


def _block_manager(num_pages: int):
  try:
    from .. import _runtime
    return _runtime.BlockManager(num_pages, PAGE)
  except ImportError:
    from .block_manager_py import BlockManager  # pure-python fallback for hosts without the build
    return BlockManager(num_pages, PAGE)


def _bucket(n: int) -> int:
  for b in (1, 2, 4, 8, 16, 24, 32, 48, 64, 96, 128, 160, 192, 256, 320, 384, 448, 512):
    if n <= b:
      return b
  return n


class ShardRunner:
  def __init__(self, config: ModelConfig, shard: Shard, device: torch.device | str = "cpu",
               weights: Optional[ShardWeights] = None, num_pages: Optional[int] = None, max_batch: int = 128,
               max_ctx: int = 4096, kv_mem_fraction: float = 0.85, seed: int = 0, use_graphs: Optional[bool] = None):
    self.config = config
    self.shard = shard
    self.device = torch.device(device)
    if self.device.type == "cuda":
      torch.cuda.set_device(self.device)
    self._random_weights, self._seed = weights is None, seed
    self.weights = weights if weights is not None else random_weights(config, shard, self.device, seed=seed)
    if self.device.type == "cuda" and os.environ.get("XOT_SHUFFLE", "1") == "1":
      # projection weights -> pre-shuffled MFMA-fragment layout: gemm_stream for decode-shaped M, gemm_big
      # (256 x 256 LDS-DMA tiles, fused SiLU / residual epilogues) for large decode batches and prefill
      # chunks -- every projection runs on the library's own kernels (XOT_ROWMAJOR_PROJ=gu,... keeps the
      # named projections row-major for A/B runs against the vendor GEMM)
      env = os.environ.get("XOT_ROWMAJOR_PROJ")
      keep = [p for p in env.split(",") if p] if env is not None else []
      # XOT_WEIGHT_DTYPE=fp8: weight-only e4m3 projections (half the bytes per decode step; opt-in, the
      # serving default and every benchmark headline stay bf16)
      self.weight_dtype = os.environ.get("XOT_WEIGHT_DTYPE", "bf16")
      prepare_for_decode(self.weights, keep_rowmajor=keep, fp8=self.weight_dtype == "fp8")
    n_layers = shard.get_layer_count()
    per_page = KVCache.bytes_per_page(config, n_layers)
    if num_pages is None:
      if self.device.type == "cuda":
        free, _ = torch.cuda.mem_get_info(self.device)
        reserve = 4 << 30  # activations, workspaces, graphs
        num_pages = int(max(free - reserve, per_page * 64) * kv_mem_fraction) // per_page
      else:
        num_pages = max(64, (max_batch * max_ctx) // PAGE // 4)
      num_pages = min(num_pages, max_batch * (-(-max_ctx // PAGE)) + 16)
    self.kv = KVCache(config, n_layers, num_pages, self.device)
    self.bm = _block_manager(num_pages)
    self.max_ctx = max_ctx
    self.max_batch = max_batch
    self.width = -(-max_ctx // PAGE)
    self.model = ShardModel(self.weights, self.kv, max_batch=max_batch, max_ctx=max_ctx)
    if use_graphs is None:
      # MoE routing runs on the device too (moe_route + grouped GEMMs), so every model is capturable
      use_graphs = self.device.type == "cuda" and os.environ.get("XOT_GRAPHS", "1") == "1"
    self.use_graphs = use_graphs
    self._graphs: Dict[tuple, dict] = {}
    # decode graphs per (batch bucket, block-table width class): a step whose longest context fits a narrower
    # table replays a graph captured with it, so the split-KV partitioning (chosen from the table width,
    # static per graph) follows the contexts actually served instead of max_ctx -- at max_ctx 8192 and
    # contexts of a few hundred tokens the full width split every sequence into 4 mostly empty partitions
    # plus a merge pass
    # (16 pages: the widest table the 8-wave single-partition attention takes at small batch, ops/kernels.py)
    self._widths = sorted({w for w in (8, 16, 32) if w < self.width} | {self.width})
    # host staging of the step inputs, double-buffered: a step's async copies read one set while the host
    # fills the other for the next step, so the host can queue a step behind the one still copying (with
    # one set it had to wait for the previous step's copies before writing the next step's inputs)
    bmax = _bucket(max_batch)
    self._sets = []
    for _ in range(2):
      st = {"tables": torch.zeros(max_batch, self.width, dtype=torch.int32),
            "ctx": torch.zeros(max_batch, dtype=torch.int32),
            "pos": torch.zeros(bmax, dtype=torch.int32),  # decode-step positions / slots (graph inputs)
            "slots": torch.zeros(bmax, dtype=torch.int64)}
      if self.device.type == "cuda":
        # pinned: an async copy out of pageable memory may wait for the stream to drain, i.e. for the step
        # already running, which would forbid queueing the next decode step behind it
        st = {k: v.pin_memory() for k, v in st.items()}
      st["cls"] = {}  # narrower block tables per width class
      st["event"] = None  # completion of the last async H2D copy out of this set
      self._sets.append(st)
    self._set_idx = 1
    self._use_set(0)

  def _use_set(self, i: int) -> None:
    st = self._sets[i]
    self._set_idx = i
    self._tables_host, self._ctx_host, self._pos_host, self._slots_host = st["tables"], st["ctx"], st["pos"], st["slots"]
    self._tables_cls = st["cls"]

  def _reuse_staging(self) -> None:
    """Switch to the other staging set; wait only if ITS last async copy (two steps back) is still running."""
    i = self._set_idx ^ 1
    ev = self._sets[i]["event"]
    if ev is not None:
      ev.synchronize()
      self._sets[i]["event"] = None
    self._use_set(i)

  def _mark_staged(self) -> None:
    if self.device.type == "cuda":
      ev = torch.cuda.Event()
      ev.record()
      self._sets[self._set_idx]["event"] = ev

  # ------------------------------------------------------------------ bookkeeping
  def has(self, rid: str) -> bool:
    return self.bm.has(rid)

  def num_tokens(self, rid: str) -> int:
    return self.bm.num_tokens(rid) if self.bm.has(rid) else 0

  def free(self, rid: str) -> None:
    self.bm.free(rid)

  def can_admit(self, rid: str, n_new: int) -> bool:
    return self.bm.can_append(rid, n_new) and self.num_tokens(rid) + n_new <= self.max_ctx

  def truncate(self, rid: str, n: int) -> None:
    self.bm.truncate(rid, n)

  # ------------------------------------------------------------------ step inputs
  def _prepare(self, rids: Sequence[str], qlens: Sequence[int]) -> StepInputs:
    if len(rids) > self.max_batch:
      raise ValueError(f"batch {len(rids)} exceeds max_batch {self.max_batch}")
    self._reuse_staging()
    pos: List[int] = []
    slots: List[int] = []
    cu = [0]
    for rid, n in zip(rids, qlens):
      start = self.num_tokens(rid)
      if start + n > self.max_ctx:
        raise ValueError(f"request {rid}: context {start + n} exceeds max_ctx {self.max_ctx}")
      slots += self.bm.append(rid, n)
      pos += self.model.rope_pos(start, n)
      cu.append(cu[-1] + n)
    B = len(rids)
    self.bm.fill_batch(list(rids), self._tables_host[:B].numpy(), self._ctx_host[:B].numpy())
    dev = self.device
    nb = non_blocking = dev.type == "cuda"
    inp = StepInputs(
      positions=torch.tensor(pos, dtype=torch.int32).to(dev, non_blocking=nb),
      slots=torch.tensor(slots, dtype=torch.int64).to(dev, non_blocking=nb),
      block_tables=self._tables_host[:B].to(dev, non_blocking=non_blocking),
      ctx_lens=self._ctx_host[:B].to(dev, non_blocking=non_blocking),
      cu_q=torch.tensor(cu, dtype=torch.int32).to(dev, non_blocking=nb),
      last_idx=torch.tensor([c - 1 for c in cu[1:]], dtype=torch.int64).to(dev, non_blocking=nb),
      max_qlen=max(qlens),
      decode=all(q == 1 for q in qlens),
    )
    self._mark_staged()
    return inp

  # ------------------------------------------------------------------ forward
  def forward(self, rids: Sequence[str], qlens: Sequence[int], x: torch.Tensor,
              image_embeds: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Run this shard for the given requests.  x = token ids [sum(qlens)] (first shard) or hidden
    [sum(qlens), D].  Allocates KV slots for the new tokens.  Returns hidden [T, D] or, on the last
    shard, fp32 logits [len(rids), V] of each request's last token.  image_embeds (LLaVA, first shard):
    projected image features for the image-token rows of x, in order."""
    x = x.to(self.device, non_blocking=True)
    if self.use_graphs and image_embeds is None and all(q == 1 for q in qlens) and len(rids) <= self.max_batch:
      return self._decode_graph(rids, x)
    inp = self._prepare(rids, qlens)
    if image_embeds is not None:
      inp.image_embeds = image_embeds.to(self.device)
    return self.model.forward(x, inp)

  def image_features(self, pixels: torch.Tensor) -> torch.Tensor:
    """LLaVA first shard: [N, 3, S, S] pixel batch -> [N * image tokens, D] projected features."""
    from ..models.vision import image_features
    if self.weights.vision is None:
      raise ValueError(f"{self.shard.model_id}: this shard has no vision tower")
    with torch.inference_mode():
      return image_features(self.config, self.weights.vision, pixels.to(self.device))

  # ------------------------------------------------------------------ graphs
  def _tables_staging(self, w: int) -> torch.Tensor:
    if w == self.width:
      return self._tables_host
    t = self._tables_cls.get(w)
    if t is None:
      t = torch.zeros(self.max_batch, w, dtype=torch.int32)
      if self.device.type == "cuda":
        t = t.pin_memory()
      self._tables_cls[w] = t
    return t

  def _decode_graph(self, rids: Sequence[str], x: torch.Tensor) -> torch.Tensor:
    B = len(rids)
    Bp = min(_bucket(B), self.max_batch)
    # host bookkeeping -> static buffers
    self._reuse_staging()
    pos, slots = [], []
    most = 0
    for rid in rids:
      start = self.num_tokens(rid)
      if start + 1 > self.max_ctx:
        raise ValueError(f"request {rid}: context exceeds max_ctx {self.max_ctx}")
      slots += self.bm.append(rid, 1)
      pos += self.model.rope_pos(start, 1)
      most = max(most, start + 1)
    need = -(-most // PAGE)
    w = next(c for c in self._widths if c >= need)
    g = self._graphs.get((Bp, w))
    if g is None:
      g = self._capture(Bp, w)
    tables = self._tables_staging(w)
    self.bm.fill_batch(list(rids), tables[:B].numpy(), self._ctx_host[:B].numpy())
    pad = Bp - B
    self._pos_host[:Bp] = torch.tensor(pos + [0] * pad, dtype=torch.int32)
    self._slots_host[:Bp] = torch.tensor(slots + [-1] * pad, dtype=torch.int64)
    g["pos"].copy_(self._pos_host[:Bp], non_blocking=True)
    g["slots"].copy_(self._slots_host[:Bp], non_blocking=True)
    self._ctx_host[B:Bp] = 0
    g["tables"].copy_(tables[:Bp], non_blocking=True)
    g["ctx"].copy_(self._ctx_host[:Bp], non_blocking=True)
    self._mark_staged()
    if self.shard.is_first_layer():
      g["x"][:B].copy_(x.view(-1).to(torch.int32))
      if pad:
        g["x"][B:].zero_()
    else:
      g["x"][:B].copy_(x)
    g["graph"].replay()
    out = g["out"]
    return tuple(t[:B] for t in out) if isinstance(out, tuple) else out[:B]

  # ------------------------------------------------------------------ split LM head
  def head_tail(self, rows_from: int) -> Optional[torch.Tensor]:
    """LM-head rows [rows_from, V) in the device layout, for a first stage that applies them to the
    normed hidden state the last stage sends (parallel/pipeline.py).  None when they cannot be derived
    here (externally loaded weights without the head on this shard)."""
    from ..models.weights import random_head_rows
    w = self.weights
    c = self.config
    if w.lm_head is not None:
      full = w.lm_head
    elif c.tie_word_embeddings and w.embed is not None:
      full = w.embed
    elif self._random_weights:
      full = None
    else:
      return None
    if full is not None:
      t = full[rows_from:]
      if linear_mod.layout_of(full) == "stream":  # rows [r, V) of the shuffled layout: a storage suffix
        t.xot_layout = "stream"
        return t
      return linear_mod.to_stream_layout(t.contiguous())
    t = random_head_rows(c, rows_from, self.device, seed=self._seed)
    return linear_mod.to_stream_layout(t)

  def _capture(self, Bp: int, w: Optional[int] = None) -> dict:
    dev = self.device
    c = self.config
    w = w or self.width
    g = {
      "pos": torch.zeros(Bp, dtype=torch.int32, device=dev),
      "slots": torch.full((Bp,), -1, dtype=torch.int64, device=dev),
      "tables": torch.zeros(Bp, w, dtype=torch.int32, device=dev),
      "ctx": torch.zeros(Bp, dtype=torch.int32, device=dev),
      "cu": torch.arange(Bp + 1, dtype=torch.int32, device=dev),
      "last": torch.arange(Bp, dtype=torch.int64, device=dev),
    }
    if self.shard.is_first_layer():
      g["x"] = torch.zeros(Bp, dtype=torch.int32, device=dev)
    else:
      g["x"] = torch.zeros(Bp, c.hidden_size, dtype=torch.bfloat16, device=dev)
    inp = StepInputs(g["pos"], g["slots"], g["tables"], g["ctx"], g["cu"], g["last"], 1, True)
    # warm up eagerly (also settles the GEMM policy for these shapes) on a side stream
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
      for _ in range(2):
        self.model.forward(g["x"], inp)
    torch.cuda.current_stream(dev).wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    linear_mod.policy.capturing = True
    try:
      # thread-local capture: the process-group watchdog thread keeps polling its RCCL events while
      # this thread captures (global mode would make those queries fail)
      with torch.cuda.graph(graph, capture_error_mode="thread_local"):
        g["out"] = self.model.forward(g["x"], inp)
    finally:
      linear_mod.policy.capturing = False
    g["graph"] = graph
    self._graphs[(Bp, w)] = g
    return g

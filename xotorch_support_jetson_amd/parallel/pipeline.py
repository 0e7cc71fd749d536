"""Ring pipeline over GPU peers: each rank holds one layer shard; M micro-batches of requests circulate
first stage -> ... -> last stage -> first stage, one ring trip per generated token (the reference's
ring, node.py:109-147 / 424-443, moved onto RCCL p2p over xGMI).

With M >= number of stages every GPU works on a different micro-batch at any moment, so whole-node
tokens/s scales with the stage count while single-request latency stays one ring trip per token.

The ring runs at the pace of its slowest stage, and the last stage also carries the final norm, the
LM head (1.07 TFLOP at 512 sequences for Llama-3's 128k vocab) and the sampler: about one extra
layer's worth of work, 10 % of a 10-layer stage at 8 GPUs.  With `split_head` (default for world > 1)
the head is split by vocab rows between the last and the first stage:
  last stage:  logits of rows [0, Vs) -> its top-k (value, index) candidates; sends the normed hidden
               state [B, D] bf16 + the candidates [B, 64] to the first stage
  first stage: logits of rows [Vs, V) into [B, 64 + V - Vs] behind the received candidates, samples
               once over that row (the global top-k lies inside it) and maps the column back to a token
so each end of the ring carries part of the head: the last stage 65 % of the rows (HEAD_SPLIT), since the first
also embeds and samples -- at 512 sequences of Llama-3-70B that evens the two ends (10.54 / 10.95 ms per tick at
70 %, 11.38 / 11.05 at 50 %, against 10.41 for a middle stage; profiles/r4/scale/headsplit_*.json).  Without it, the last stage samples and sends the
ids [B] int32.  Transfers are only these tensors; positions and masks live on the devices.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import torch

from ..ops import kernels as K
from ..ops.linear import linear
from ..runtime.runner import ShardRunner

KC = 64  # candidate slots per row in the split-head hand-off (>= top_k)
HEAD_SPLIT = 0.65  # default fraction of the LM-head rows on the last stage (measured balance, profiles/r4/scale/)

# tokens per prefill forward of RingStage (whole sequences): the tall GEMMs' M (XOT_PREFILL_CHUNK)
PREFILL_CHUNK = int(os.environ.get("XOT_PREFILL_CHUNK", "8192"))


@dataclass
class MicroBatch:
  rids: List[str]
  prompt: Optional[torch.Tensor] = None  # [B, L] int32 (first stage)
  temps: Optional[torch.Tensor] = None  # [B] fp32 (the sampling stage)
  tokens: List[List[int]] = field(default_factory=list)  # generated ids (the sampling stage)


class RingStage:
  """One rank's role in the ring.  `transport` provides isend/irecv to neighbours (RCCL, gloo or loopback).

  Hand-off from the last stage to the first ("item"): the sampled ids [B] int32, or with the split head
  the tuple (normed hidden [B, D] bf16, candidate values [B, KC] fp32, candidate ids [B, KC] int32)."""

  def __init__(self, runner: ShardRunner, rank: int, world: int, transport, top_k: int = 35, seed: int = 1234,
               split_head: Optional[bool] = None):
    self.r = runner
    self.rank, self.world = rank, world
    self.t = transport
    self.first = runner.shard.is_first_layer()
    self.last = runner.shard.is_last_layer()
    self.prev = (rank - 1) % world
    self.next = (rank + 1) % world
    self.top_k = top_k
    dev = runner.device
    self.seed_off = torch.tensor([seed, 0], dtype=torch.int64, device=dev)
    self.D = runner.config.hidden_size
    V = runner.config.vocab_size
    # rows of the last stage's share (GEMM-tile aligned).  XOT_HEAD_SPLIT: its fraction of the vocab -- the first
    # stage also runs the embedding, the candidate copy and the sampler over its columns, so a share above one
    # half evens the two ends out
    frac = float(os.environ.get("XOT_HEAD_SPLIT", str(HEAD_SPLIT)))
    self.vs = int(V * frac) // 256 * 256
    want = os.environ.get("XOT_SPLIT_HEAD", "1") == "1" if split_head is None else split_head
    # the decision depends only on config and arguments, so every rank takes the same one
    self.split = bool(want and world > 1 and 0 < self.vs < V and 1 <= top_k <= KC and top_k < self.vs)
    self.head_tail = None
    if self.split and self.first:
      self.head_tail = runner.head_tail(self.vs)
      if self.head_tail is None:
        raise ValueError("split LM head: the first stage cannot derive LM-head rows for externally loaded "
                         "weights; pass split_head=False")
    if self.split and self.last:
      runner.model.head_rows = self.vs
    self.samples = self.first if self.split else self.last  # the stage that draws the tokens

  # ---------------------------------------------------------------- sampling / hand-off
  def _sample(self, logits: torch.Tensor, temps: torch.Tensor) -> torch.Tensor:
    tok = K.sample(logits, temps, self.top_k, self.seed_off)
    self.seed_off[1] += 1
    return tok

  def _head_part(self, y) -> tuple:
    """Last stage, split head: (logits of rows [0, Vs), normed hidden) -> hand-off item."""
    logits, xn = y
    vals, idx = K.topk_cand(logits, self.top_k, KC)
    return xn.contiguous().clone(), vals, idx  # clone: xn may be a decode graph's static buffer

  def _send_item(self, item) -> None:
    if isinstance(item, tuple):
      for t in item:
        self.t.isend(t, self.next)
    else:
      self.t.isend(item, self.next)

  def _finish_head(self, xn: torch.Tensor, vals: torch.Tensor, idx: torch.Tensor, temps: torch.Tensor) -> torch.Tensor:
    """First stage, split head: logits of rows [Vs, V) behind the received candidates, one sampler pass."""
    B = xn.shape[0]
    V = self.r.config.vocab_size
    buf = torch.empty(B, KC + V - self.vs, dtype=torch.float32, device=xn.device)
    buf[:, :KC].copy_(vals)
    linear(xn, self.head_tail, out=buf[:, KC:], out_dtype=torch.float32)
    j = self._sample(buf, temps).long()
    cand = idx.long().gather(1, j.clamp(max=KC - 1).unsqueeze(1)).squeeze(1)
    return torch.where(j < KC, cand, j - KC + self.vs).to(torch.int32)

  def _recv_item(self, B: int) -> tuple:
    """First stage, split head: receive the last stage's hand-off (normed hidden, candidates) of B rows."""
    dev = self.r.device
    xn = torch.empty(B, self.D, dtype=torch.bfloat16, device=dev)
    vals = torch.empty(B, KC, dtype=torch.float32, device=dev)
    idx = torch.empty(B, KC, dtype=torch.int32, device=dev)
    works = [self.t.irecv(xn, self.prev), self.t.irecv(vals, self.prev), self.t.irecv(idx, self.prev)]
    for w in works:
      self.t.wait(w)
    return xn, vals, idx

  def _recv_and_sample(self, mb: MicroBatch) -> torch.Tensor:
    return self._finish_head(*self._recv_item(len(mb.rids)), mb.temps)

  # ---------------------------------------------------------------- per-tick device timing (bench diagnostics)
  def start_timing(self) -> None:
    """Record (start, data in, done) events on the compute stream around every decode tick from now on:
    data-in minus start is the time the stream sat waiting for the previous stage's hand-off (the recv
    wait), done minus data-in the stage's own work (layers, head share, sampling)."""
    self._events = []

  def timing(self) -> dict:
    """Per-tick means (ms) of the recorded ticks: {'ticks', 'stage_ms', 'recv_wait_ms'}; syncs the device."""
    ev = getattr(self, "_events", None) or []
    if not ev:
      return {"ticks": 0, "stage_ms": None, "recv_wait_ms": None}
    if self.r.device.type == "cuda":
      torch.cuda.synchronize(self.r.device)
    wait = sum(a.elapsed_time(b) for a, b, _ in ev) / len(ev)
    work = sum(b.elapsed_time(c) for _, b, c in ev) / len(ev)
    return {"ticks": len(ev), "stage_ms": round(work, 3), "recv_wait_ms": round(wait, 3)}

  def _mark(self):
    if getattr(self, "_events", None) is None or self.r.device.type != "cuda":
      return None
    e = torch.cuda.Event(enable_timing=True)
    e.record()
    return e

  # ---------------------------------------------------------------- one micro-batch through this stage
  def prefill(self, mb: MicroBatch, chunk_tokens: int = 0):
    """Run the prompts of a micro-batch through this stage in chunks of whole sequences.  First stage
    reads mb.prompt; others receive hidden states.  The last stage returns the hand-off item of the
    first generated token (the sampled ids [B], or the split-head tuple); other stages None."""
    B, L = len(mb.rids), (mb.prompt.shape[1] if mb.prompt is not None else 0)
    dev = self.r.device
    chunk_tokens = chunk_tokens or PREFILL_CHUNK
    per = max(1, chunk_tokens // max(L, 1)) if L else B
    outs = []
    for lo in range(0, B, per):
      rids = mb.rids[lo:lo + per]
      n = len(rids)
      if self.first:
        x = mb.prompt[lo:lo + n].reshape(-1).to(dev)
        Lc = mb.prompt.shape[1]
      else:
        meta = torch.empty(1, dtype=torch.int64, device=dev)
        self.t.recv(meta, self.prev)
        Lc = int(meta.item())
        x = torch.empty(n * Lc, self.D, dtype=torch.bfloat16, device=dev)
        self.t.recv(x, self.prev)
      y = self.r.forward(rids, [Lc] * n, x)
      if not self.last:
        meta = torch.tensor([Lc], dtype=torch.int64, device=dev)
        self.t.isend(meta, self.next)
        self.t.isend(y.contiguous(), self.next)
      elif self.split:
        outs.append(self._head_part(y))
      else:
        outs.append(self._sample(y, mb.temps[lo:lo + n]))
    if not self.last:
      return None
    if self.split:
      return tuple(torch.cat([o[i] for o in outs]) for i in range(3))
    return torch.cat(outs)

  def decode_tick(self, mb: MicroBatch, item_in=None, send: bool = True):
    """One decode step for one micro-batch on this stage.  item_in: the hand-off item when this stage
    is the whole ring (world 1); otherwise the first stage receives it from the last.  Returns
    (sampled ids or None, hand-off item produced here or None)."""
    B = len(mb.rids)
    dev = self.r.device
    sampled = None
    e0 = self._mark()
    if self.first:
      if item_in is not None:
        x = item_in
        e1 = e0
      elif self.split:
        got = self._recv_item(B)
        e1 = self._mark()
        x = sampled = self._finish_head(*got, mb.temps)
      else:
        x = torch.empty(B, dtype=torch.int32, device=dev)
        self.t.wait(self.t.irecv(x, self.prev))
        e1 = self._mark()
    else:
      x = torch.empty(B, self.D, dtype=torch.bfloat16, device=dev)
      self.t.wait(self.t.irecv(x, self.prev))
      e1 = self._mark()
    y = self.r.forward(mb.rids, [1] * B, x)
    if not self.last:
      # y is the decode graph's static output buffer: the next replay overwrites it, so hand RCCL a copy
      self.t.isend(y.clone(), self.next)
      if e0 is not None:
        self._events.append((e0, e1, self._mark()))
      return sampled, None
    item = self._head_part(y) if self.split else self._sample(y, mb.temps)
    if not self.split:
      sampled = item
    if self.world > 1 and send:
      self._send_item(item)
    if e0 is not None:
      self._events.append((e0, e1, self._mark()))
    return sampled, item


def run_decode_steps(stage: RingStage, mbs: Sequence[MicroBatch], steps: int, first_tokens=None,
                     record: bool = False):
  """`steps` ring rounds: every micro-batch advances one token per round.  first_tokens: the hand-off
  items the last stage holds from prefill or from the previous call (for world == 1 that is this
  stage).  In the final round the last stage keeps its items (nobody would consume another ring
  trip) and returns them, to seed the next call.  With the split head a round's tokens are drawn by
  the first stage at the start of the next round, so the first call yields steps tokens per sequence
  (the prefill token included) instead of steps + 1."""
  local = list(first_tokens) if (first_tokens is not None and stage.world == 1) else None
  pending: List[Optional[object]] = [None] * len(mbs)
  if stage.last and stage.world > 1 and first_tokens is not None:
    for item in first_tokens:  # hand the held items to the first stage to start the ring
      stage._send_item(item)
  for s in range(steps):
    final_round = s == steps - 1
    for m, mb in enumerate(mbs):
      sampled, item = stage.decode_tick(mb, local[m] if local is not None else None, send=not final_round)
      if sampled is not None and record:
        mb.tokens.append(sampled.tolist())
      if item is not None:
        pending[m] = item
        if local is not None:
          local[m] = item
  return pending if stage.last else None

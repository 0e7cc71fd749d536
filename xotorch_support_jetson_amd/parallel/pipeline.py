"""Ring pipeline over GPU peers: each rank holds one layer shard; M micro-batches of requests circulate
first stage -> ... -> last stage (samples on device) -> first stage, one ring trip per generated token
(the reference's ring, node.py:109-147 / 424-443, moved onto RCCL p2p over xGMI).

With M >= number of stages every GPU works on a different micro-batch at any moment, so whole-node
tokens/s scales with the stage count while single-request latency stays one ring trip per token.
Transfers: hidden [B, D] bf16 between stages, sampled ids [B] int32 from last to first — nothing else.
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import torch

from ..ops import kernels as K
from ..runtime.runner import ShardRunner


@dataclass
class MicroBatch:
  rids: List[str]
  prompt: Optional[torch.Tensor] = None  # [B, L] int32 (first stage)
  temps: Optional[torch.Tensor] = None  # [B] fp32 (last stage)
  tokens: List[List[int]] = field(default_factory=list)  # generated ids (last stage)


class RingStage:
  """One rank's role in the ring.  `transport` provides isend/irecv to neighbours (RCCL, gloo or loopback)."""

  def __init__(self, runner: ShardRunner, rank: int, world: int, transport, top_k: int = 35, seed: int = 1234):
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

  # ---------------------------------------------------------------- one micro-batch through this stage
  def _sample(self, logits: torch.Tensor, temps: torch.Tensor) -> torch.Tensor:
    tok = K.sample(logits, temps, self.top_k, self.seed_off)
    self.seed_off[1] += 1
    return tok

  def prefill(self, mb: MicroBatch, chunk_tokens: int = 8192) -> Optional[torch.Tensor]:
    """Run the prompts of a micro-batch through this stage in chunks of whole sequences.  First stage
    reads mb.prompt; others receive hidden states.  Last stage returns the first sampled ids [B]."""
    B, L = len(mb.rids), (mb.prompt.shape[1] if mb.prompt is not None else 0)
    dev = self.r.device
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
      else:
        outs.append(self._sample(y, mb.temps[lo:lo + n]))
    if self.last:
      return torch.cat(outs)
    return None

  def decode_tick(self, mb: MicroBatch, tokens_in: Optional[torch.Tensor] = None,
                  send_tokens: bool = True) -> Optional[torch.Tensor]:
    """One decode step for one micro-batch on this stage.  First stage: ids come from `tokens_in`
    (single-stage ring) or from the last stage; last stage returns the sampled ids."""
    B = len(mb.rids)
    dev = self.r.device
    if self.first:
      if tokens_in is None:
        tokens_in = torch.empty(B, dtype=torch.int32, device=dev)
        self.t.irecv(tokens_in, self.prev).wait()
      x = tokens_in
    else:
      x = torch.empty(B, self.D, dtype=torch.bfloat16, device=dev)
      self.t.irecv(x, self.prev).wait()
    y = self.r.forward(mb.rids, [1] * B, x)
    if self.last:
      tok = self._sample(y, mb.temps)
      if self.world > 1 and send_tokens:
        self.t.isend(tok, self.next)
      return tok
    # y is the decode graph's static output buffer: the next replay overwrites it, so hand RCCL a copy
    self.t.isend(y.clone(), self.next)
    return None


def run_decode_steps(stage: RingStage, mbs: Sequence[MicroBatch], steps: int,
                     first_tokens: Optional[List[torch.Tensor]] = None, record: bool = False):
  """`steps` ring rounds: every micro-batch advances one token per round.  first_tokens are the ids
  produced by prefill or by the previous call (held by the last stage; for world==1 that is this
  stage).  Returns the ids sampled in the final round (last stage), to seed the next call."""
  local = list(first_tokens) if (first_tokens is not None and stage.world == 1) else None
  last_toks: List[Optional[torch.Tensor]] = [None] * len(mbs)
  if stage.last and stage.world > 1 and first_tokens is not None:
    for tok in first_tokens:  # hand the prefill tokens to the first stage to start the ring
      stage.t.isend(tok, stage.next)
  for s in range(steps):
    final_round = s == steps - 1
    for m, mb in enumerate(mbs):
      # in the final round the last stage keeps its ids: nobody would consume another ring trip
      tok = stage.decode_tick(mb, local[m] if local is not None else None, send_tokens=not final_round)
      if tok is not None:
        last_toks[m] = tok
        if local is not None:
          local[m] = tok
        if record:
          mb.tokens.append(tok.tolist())
  return last_toks if stage.last else None

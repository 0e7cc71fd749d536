"""Pipeline-parallel training over the GPU ring (RCCL send/recv over xGMI; gloo on CPU hosts).

The device-native form of the reference's SendExample training protocol
(xotorch/orchestration/node.py:299-345, grpc_peer_handle.py:138-159): rank r holds layer shard r as a
ShardTrainer (HIP RMSNorm / SiLU / RoPE / cross-entropy kernels + fused AdamW, hipBLASLt GEMMs).
One optimizer step = GPipe schedule over M micro-batches:

  forward phase   for i in 0..M-1: recv act_i from r-1 (or embed ids) -> forward (autograd graph kept)
                                   -> send act_i to r+1;  the last stage computes the loss of act_i
  backward phase  for i in 0..M-1: recv grad_i from r+1 (last stage: d loss_i) -> backward
                                   -> send d act_i to r-1
  step            global grad-norm (all-reduce of squared norms) -> AdamW on every stage

or (schedule="1f1b") the one-forward-one-backward order: rank r runs min(M, world - r - 1) warm-up
forwards, then alternates F(i + warm-up) / B(i), then drains the remaining backwards.  Same gradients
and the same bubble as GPipe, but at most world - r micro-batches' autograd graphs are alive on rank r
instead of M, so long sequences / many micro-batches fit.  Upstream ranks always run further ahead,
so a rank never blocks on a gradient whose producer is waiting for an activation it has not sent
(activations and gradients travel on separate per-direction communicators, see comm.P2PTransport).

Every rank issues its p2p operations in the same micro-batch order, so the per-communicator FIFO of
RCCL never blocks a send behind a receive its peer has not posted.  Activations and gradients are
bf16 [mb, L, D]; the loss is normalised by the global number of target tokens, so accumulated
gradients equal those of one big batch.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional

import torch
import torch.distributed as dist

from ..train.trainer import ShardTrainer


@dataclass
class TrainBatch:
  x: torch.Tensor  # [mb, L] int token ids (used by the first stage)
  y: torch.Tensor  # [mb, L] int targets (used by the last stage)
  lengths: torch.Tensor  # [mb] valid target tokens per row


class PipelineTrainer:
  def __init__(self, trainer: ShardTrainer, rank: int, world: int, transport, schedule: str = "gpipe"):
    assert schedule in ("gpipe", "1f1b"), schedule
    self.schedule = schedule
    self.tr = trainer
    self.rank, self.world = rank, world
    self.t = transport
    self.first = trainer.shard.is_first_layer()
    self.last = trainer.shard.is_last_layer()
    self.prev, self.next = rank - 1, rank + 1
    self.D = trainer.c.hidden_size
    self.dev = trainer.device
    # tied input/output embeddings split over the first and last stage: their gradients are summed
    # over a 2-rank group so both copies take the same update
    self.tied_group = None
    if world > 1 and trainer.c.tie_word_embeddings:
      self.tied_group = dist.new_group([0, world - 1])  # every rank takes part in group creation
    self.tied_name = "embed" if self.first else ("lm_head" if self.last else None)

  def _reduce_sq(self, t: torch.Tensor) -> torch.Tensor:
    if self.world > 1:
      t = t.to(self.dev)
      dist.all_reduce(t)
    return t

  def _fwd(self, b: TrainBatch):
    """Forward of one micro-batch (autograd graph kept); hands the activation to the next stage."""
    mb, L = b.x.shape
    if self.first:
      inp = b.x.to(self.dev)
    else:
      inp = torch.empty(mb, L, self.D, dtype=torch.bfloat16, device=self.dev)
      self.t.wait(self.t.irecv(inp, self.prev))
    leaf, out = self.tr.forward_train(inp)
    if not self.last:
      self.t.isend(out.detach().contiguous(), self.next)
    return leaf, out

  def _bwd(self, b: TrainBatch, saved, denom: float, losses: list) -> None:
    """Backward of one micro-batch (loss on the last stage, else the gradient from the next stage);
    hands d(input) to the previous stage."""
    leaf, out = saved
    if self.last:
      loss, gin = self.tr.backward_accumulate(leaf, out, target=b.y, length=b.lengths, denom=denom)
      losses.append(loss)
    else:
      g = torch.empty_like(out, dtype=torch.bfloat16)
      self.t.wait(self.t.irecv(g, self.next))
      _, gin = self.tr.backward_accumulate(leaf, out, grad_out=g)
    if not self.first:
      self.t.isend(gin.to(torch.bfloat16).contiguous(), self.prev)

  def step(self, batches: List[TrainBatch]) -> Optional[float]:
    """One optimizer step over the micro-batches; returns the mean loss on the last stage (None
    elsewhere; also broadcast to rank 0 when world > 1)."""
    tr = self.tr
    tr.zero_grad()
    denom = float(sum(int(b.lengths.sum()) for b in batches))
    saved = {}
    losses = []
    M = len(batches)
    if self.schedule == "1f1b":
      warm = min(M, self.world - self.rank - 1)
      for i in range(warm):
        saved[i] = self._fwd(batches[i])
      for i in range(M - warm):
        saved[i + warm] = self._fwd(batches[i + warm])
        self._bwd(batches[i], saved.pop(i), denom, losses)
      for i in range(M - warm, M):
        self._bwd(batches[i], saved.pop(i), denom, losses)
    else:
      for i, b in enumerate(batches):
        saved[i] = self._fwd(b)
      for i, b in enumerate(batches):
        self._bwd(b, saved.pop(i), denom, losses)
    self.t.drain()
    grads = None
    if self.tied_group is not None and self.tied_name is not None:
      # the local gradient of this stage's copy: on the GPU it may sit in a GradAcc buffer (fp32 embedding
      # index-add, fused-CE dHead), which tr.grads() prefers over p.grad -- sum THAT over the two ends in fp32
      # and hand the sum to the optimizer as it is (no bf16 rounding on one end only), so both copies take
      # bit-identical updates
      name = self.tied_name
      grads = tr.grads()
      g = grads.get(name)
      g = torch.zeros_like(tr.params[name], dtype=torch.float32) if g is None else g.float()
      dist.all_reduce(g, group=self.tied_group)
      grads[name] = g
    tied_copy = ("lm_head",) if (self.tied_group is not None and self.last) else ()
    tr.apply(self._reduce_sq, norm_exclude=tied_copy, grads=grads)
    loss = float(torch.stack(losses).sum()) if losses else None
    if self.world > 1:
      lt = torch.tensor([loss if loss is not None else 0.0], dtype=torch.float32, device=self.dev)
      dist.all_reduce(lt)  # only the last stage contributes
      loss = float(lt)
    return loss

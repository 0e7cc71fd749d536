"""Data-parallel training: one full model replica per GPU, gradients summed by bucketed all-reduce
overlapped with the backward pass.

MI355X-first alternative to the reference's only strategy (layer pipeline): with
288 GB of HBM per GPU a Llama-3-8B replica with fp32 master weights and AdamW moments (~128 GB) fits on
every device, so instead of a GPipe pipeline with its (N-1)/(M+N-1) bubble each GPU runs the whole
model on its own micro-batches and the only traffic is one all-reduce of the gradients per step.

Schedule of one optimizer step (each rank its own micro-batches, loss normalised by the GLOBAL target
token count so the summed gradients equal one big batch's):
  forward + backward of micro-batches 0..M-2       gradients accumulate in bf16 (projections inside
                                                   their backward GEMM, the rest in .grad)
  backward of the last micro-batch                 accumulation hooks copy each finished
                                                   gradient into its fp32 bucket; a full bucket starts
                                                   an async all-reduce (RCCL's stream) while autograd
                                                   keeps computing the earlier layers' gradients
  wait for the buckets -> global grad norm (identical on every rank, no extra reduce) -> fused AdamW
                                                   reading the fp32 buckets directly
Buckets follow reverse parameter order (the order backward produces them) and hold ~256 MB: xGMI
all-reduce rings are per-link bandwidth bound, so a few large messages beat many small ones.

Collective order.  Every rank must issue the bucket all-reduces in the same order, or RCCL pairs up
unrelated buffers (gloo aborts with a size mismatch).  The order in which buckets *fill* depends on the
rank's work (backward finishes the embedding last, a rank with no micro-batch fills nothing until the
flush), so a full bucket is only marked ready; the launcher starts buckets strictly in list order,
each as soon as it and every earlier bucket are ready.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from ..train import autograd_ops as A
from ..train.trainer import ShardTrainer
from .pipeline_train import TrainBatch


@dataclass
class _Bucket:
  names: List[str]
  flat: torch.Tensor  # fp32, all gradients of the bucket back to back
  views: Dict[str, torch.Tensor] = field(default_factory=dict)
  done: set = field(default_factory=set)
  work: Optional[object] = None
  ready: bool = False


class DataParallelTrainer:
  def __init__(self, trainer: ShardTrainer, rank: int, world: int, bucket_mb: float = 256.0, group=None):
    if not (trainer.shard.is_first_layer() and trainer.shard.is_last_layer()):
      raise ValueError("data parallelism needs the whole model on every rank")
    self.tr = trainer
    self.rank, self.world = rank, world
    self.group = group
    self.dev = trainer.device
    limit = int(bucket_mb * (1 << 20)) // 4
    self.buckets: List[_Bucket] = []
    self.bucket_of: Dict[str, int] = {}
    names = list(trainer.params)[::-1]  # backward produces the last layers' gradients first
    cur: List[str] = []
    size = 0
    for n in names + [None]:
      numel = trainer.params[n].numel() if n is not None else 0
      if cur and (n is None or size + numel > limit):
        flat = torch.zeros(size, dtype=torch.float32, device=self.dev)
        b = _Bucket(cur, flat)
        off = 0
        for m in cur:
          p = trainer.params[m]
          b.views[m] = flat[off:off + p.numel()].view_as(p)
          off += p.numel()
          self.bucket_of[m] = len(self.buckets)
        self.buckets.append(b)
        cur, size = [], 0
      if n is not None:
        cur.append(n)
        size += numel
    self._armed = False
    self._next = 0  # first bucket not yet launched (launch order == list order on every rank)
    # autograd-accumulated parameters signal through post-accumulate-grad hooks, projections with fused
    # accumulation (trainer.acc, A.LinearFn) through their GradAcc callback
    self._hooks = [p.register_post_accumulate_grad_hook(self._hook(n)) for n, p in trainer.params.items()
                   if n not in trainer.acc]
    for n, a in trainer.acc.items():
      a.cb = self._acc_cb(n)

  def _ready(self, name: str, g: torch.Tensor) -> None:
    b = self.buckets[self.bucket_of[name]]
    b.views[name].copy_(g)
    b.done.add(name)
    if len(b.done) == len(b.names):
      b.ready = True
      self._launch_ready()

  def _hook(self, name: str):
    def fn(p: torch.Tensor):
      if not self._armed or p.grad is None:
        return
      self._ready(name, p.grad)
      p.grad = None
    return fn

  def _acc_cb(self, name: str):
    def fn():
      if self._armed:
        A.join_dw_stream()  # the buffer may still be written on the weight-gradient side stream
        self._ready(name, self.tr.acc[name].buf)
    return fn

  def _launch_ready(self) -> None:
    """Start every ready bucket whose predecessors have all started (same order on every rank)."""
    while self._next < len(self.buckets) and self.buckets[self._next].ready:
      b = self.buckets[self._next]
      if self.world > 1:
        b.work = dist.all_reduce(b.flat, group=self.group, async_op=True)
      self._next += 1

  def _global_tokens(self, batches: List[TrainBatch]) -> float:
    n = torch.tensor([float(sum(int(b.lengths.sum()) for b in batches))], dtype=torch.float64)
    if self.world > 1:
      n = n.to(self.dev) if dist.get_backend(self.group) == "nccl" else n
      dist.all_reduce(n, group=self.group)
    return float(n)

  def step(self, batches: List[TrainBatch]) -> float:
    """One optimizer step over this rank's micro-batches (possibly none: the rank then contributes zero
    gradients to every bucket); returns the global mean loss (every rank)."""
    tr = self.tr
    tr.zero_grad()
    denom = self._global_tokens(batches)
    for b in self.buckets:
      b.done, b.work, b.ready = set(), None, False
    self._next = 0
    losses = []
    for i, mb in enumerate(batches):
      self._armed = i == len(batches) - 1
      leaf, out = tr.forward_train(mb.x.to(self.dev))
      loss, _ = tr.backward_accumulate(leaf, out, target=mb.y, length=mb.lengths, denom=denom)
      losses.append(loss)
      del out
    self._armed = False
    A.join_dw_stream()
    for b in self.buckets:  # parameters that received no gradient this step count as zeros
      if len(b.done) < len(b.names):
        for n in b.names:
          if n in b.done:
            continue
          p, a = tr.params[n], tr.acc.get(n)
          if a is not None and not a.fresh:
            b.views[n].copy_(a.buf)
          elif p.grad is not None:
            b.views[n].copy_(p.grad)
            p.grad = None
          else:
            b.views[n].zero_()
          b.done.add(n)
        b.ready = True
    self._launch_ready()
    assert self._next == len(self.buckets)
    for b in self.buckets:
      if b.work is not None:
        b.work.wait()
    tr.apply(grads={n: b.views[n] for b in self.buckets for n in b.names})
    loss = torch.stack(losses).sum().reshape(1).float() if losses else torch.zeros(1, device=self.dev)
    if self.world > 1:
      loss = loss.to(self.dev) if dist.get_backend(self.group) == "nccl" else loss.cpu()
      dist.all_reduce(loss, group=self.group)
    return float(loss)

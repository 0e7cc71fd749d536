"""Process-group bootstrap and point-to-point transports for the GPU ring.

One process per GPU (torchrun / `xot --gpus N` spawner).  The data plane between neighbouring
pipeline stages is RCCL send/recv over xGMI (torch.distributed backend "nccl" is RCCL on ROCm);
ops are issued as isend/irecv so RCCL's own stream carries the transfer and the compute stream only
waits on the recv event right before the tensor is consumed.  On CPU hosts (tests) the same code runs
over gloo.  A `LoopbackTransport` lets N virtual stages share one process/GPU (1-GPU ring tests).

Reference parity: replaces the gRPC SendTensor hop with the JSON-serialised mask/state
(xotorch/networking/grpc/grpc_peer_handle.py:117-136, grpc_server.py:77-92): only the activation
(bf16) or the sampled token ids (int32) cross the link; positions/masks live on the device.
"""
from __future__ import annotations

import datetime
import os
from collections import defaultdict, deque
from typing import Optional

import torch
import torch.distributed as dist

from .health import FaultInjector, HealthMonitor, wait_work


def env_rank() -> tuple[int, int, int]:
  return int(os.environ.get("RANK", 0)), int(os.environ.get("LOCAL_RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))


def init_distributed(backend: Optional[str] = None, timeout_s: int = 1800) -> tuple[int, int, torch.device]:
  """Init the default process group from torchrun-style env vars.  Returns (rank, world, device).
  XOT_DIST_BACKEND=gloo forces gloo on GPU hosts too (single-GPU rehearsals of the multi-rank ring;
  P2PTransport then stages device tensors through host memory)."""
  rank, local, world = env_rank()
  if torch.cuda.is_available():
    local = local % torch.cuda.device_count()  # more ranks than GPUs only in single-GPU rehearsals
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
  else:
    device = torch.device("cpu")
  if world > 1 and not dist.is_initialized():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    be = backend or os.environ.get("XOT_DIST_BACKEND") or ("nccl" if device.type == "cuda" else "gloo")
    kw = dict(backend=be, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=timeout_s))
    if be == "nccl":
      kw["device_id"] = device
    dist.init_process_group(**kw)
  return rank, world, device


def ring_edges(world: int) -> list:
  """Directed neighbour edges of the ring, both directions (activations forward, grads / ids back)."""
  edges = []
  for i in range(world):
    for e in ((i, (i + 1) % world), ((i + 1) % world, i)):
      if e[0] != e[1] and e not in edges:
        edges.append(e)
  return edges


class _StagedRecv:
  """irecv into a host bounce buffer (gloo cannot address device memory); wait() copies it in."""

  def __init__(self, work, host: torch.Tensor, dst: torch.Tensor):
    self.work, self.host, self.dst = work, host, dst

  def wait(self, monitor=None):
    wait_work(self.work, monitor)
    self.dst.copy_(self.host)
    return True

  def is_completed(self):
    return self.work.is_completed()


class P2PTransport:
  """Ordered tensor hand-off to/from ring neighbours.

  Every directed edge (src -> dst) gets its own 2-rank process group, i.e. its own RCCL communicator
  and stream.  With one shared communicator per rank pair, a large hand-off in one direction (8 MB of
  activations) and the opposite-direction traffic (sampled ids, or gradients in training) would be
  serialised on one stream in issue order and can wait on each other across ranks — with one stream
  per direction each link only ever carries a FIFO of same-direction messages, which cannot deadlock.
  """

  def __init__(self, rank: int, world: int, monitor: Optional[HealthMonitor] = None,
               injector: Optional[FaultInjector] = None, edges: Optional[list] = None):
    """`edges`: the directed (src, dst) pairs to give communicators (default: the ring's neighbour edges)."""
    self.rank, self.world = rank, world
    self.monitor = monitor  # parallel/health.py: host waits raise PeerFailure instead of hanging
    self.injector = injector if injector is not None else FaultInjector.from_env(rank, monitor)
    self._pending = []
    self._groups = {}
    self._staged = False
    self.sent_bytes = 0  # payload handed to isend (bench diagnostics)
    if world > 1 and dist.is_initialized():
      self._staged = dist.get_backend() == "gloo"
      for e in (edges if edges is not None else ring_edges(world)):  # every rank creates every group, in order
        self._groups[e] = dist.new_group(ranks=sorted(e))

  def _group(self, src: int, dst: int):
    return self._groups.get((src, dst))

  def isend(self, t: torch.Tensor, dst: int):
    if self.monitor is not None:
      self.monitor.check()
    if self.injector is not None:
      self.injector.before_send()
    self.sent_bytes += t.numel() * t.element_size()
    if self._staged and t.is_cuda:
      t = t.to("cpu")
    w = dist.isend(t, dst, group=self._group(self.rank, dst))
    self._pending.append((w, t))  # keep the tensor alive until the send completes
    if len(self._pending) > 64:
      self.reap()
    return w

  def irecv(self, t: torch.Tensor, src: int):
    if self._staged and t.is_cuda:
      host = torch.empty(t.shape, dtype=t.dtype)
      return _StagedRecv(dist.irecv(host, src, group=self._group(src, self.rank)), host, t)
    return dist.irecv(t, src, group=self._group(src, self.rank))

  def recv(self, t: torch.Tensor, src: int) -> torch.Tensor:
    self.wait(self.irecv(t, src))
    return t

  def wait(self, work) -> None:
    """Host wait on a recv.  gloo (and staged) waits block the host, so with a monitor they poll it and
    raise PeerFailure; an RCCL wait only orders the compute stream after the comm stream and returns at
    once (polling it would serialise host and GPU), so a dead peer there is handled by the monitor's
    communicator abort."""
    if isinstance(work, _StagedRecv):
      work.wait(self.monitor)
    elif self._staged or dist.is_initialized() and dist.get_backend() == "gloo":
      wait_work(work, self.monitor)
    else:
      work.wait()

  def reap(self):
    keep = []
    for w, t in self._pending:
      if not w.is_completed():
        keep.append((w, t))
    self._pending = keep

  def drain(self):
    for w, _ in self._pending:
      w.wait()
    self._pending = []


class _Done:
  def wait(self):
    return None

  def is_completed(self):
    return True


class LoopbackTransport:
  """N virtual stages in one process: isend appends to a per-(src,dst) queue, irecv pops from it."""

  _queues = defaultdict(deque)

  def __init__(self, rank: int, world: int):
    self.rank, self.world = rank, world
    self.sent_bytes = 0

  def isend(self, t: torch.Tensor, dst: int):
    LoopbackTransport._queues[(self.rank, dst)].append(t.clone())
    return _Done()

  def irecv(self, t: torch.Tensor, src: int):
    t.copy_(LoopbackTransport._queues[(src, self.rank)].popleft())
    return _Done()

  def recv(self, t: torch.Tensor, src: int) -> torch.Tensor:
    return self.irecv(t, src) and t

  def wait(self, work) -> None:
    work.wait()

  def reap(self):
    pass

  def drain(self):
    pass

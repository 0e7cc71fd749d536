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


def env_rank() -> tuple[int, int, int]:
  return int(os.environ.get("RANK", 0)), int(os.environ.get("LOCAL_RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))


def init_distributed(backend: Optional[str] = None, timeout_s: int = 1800) -> tuple[int, int, torch.device]:
  """Init the default process group from torchrun-style env vars.  Returns (rank, world, device)."""
  rank, local, world = env_rank()
  if torch.cuda.is_available():
    local = local % torch.cuda.device_count()  # more ranks than GPUs only in single-GPU rehearsals
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
  else:
    device = torch.device("cpu")
  if world > 1 and not dist.is_initialized():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    be = backend or ("nccl" if device.type == "cuda" else "gloo")
    kw = dict(backend=be, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=timeout_s))
    if be == "nccl":
      kw["device_id"] = device
    dist.init_process_group(**kw)
  return rank, world, device


class P2PTransport:
  """Ordered tensor hand-off to/from ring neighbours over the default process group."""

  def __init__(self, rank: int, world: int):
    self.rank, self.world = rank, world
    self._pending = []

  def isend(self, t: torch.Tensor, dst: int):
    w = dist.isend(t, dst)
    self._pending.append((w, t))  # keep the tensor alive until the send completes
    if len(self._pending) > 64:
      self.reap()
    return w

  def irecv(self, t: torch.Tensor, src: int):
    return dist.irecv(t, src)

  def recv(self, t: torch.Tensor, src: int) -> torch.Tensor:
    dist.irecv(t, src).wait()
    return t

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

  def isend(self, t: torch.Tensor, dst: int):
    LoopbackTransport._queues[(self.rank, dst)].append(t.clone())
    return _Done()

  def irecv(self, t: torch.Tensor, src: int):
    t.copy_(LoopbackTransport._queues[(src, self.rank)].popleft())
    return _Done()

  def recv(self, t: torch.Tensor, src: int) -> torch.Tensor:
    return self.irecv(t, src) and t

  def reap(self):
    pass

  def drain(self):
    pass

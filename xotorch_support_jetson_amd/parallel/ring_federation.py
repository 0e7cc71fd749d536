"""A local RCCL GPU ring as ONE peer of a discovered cluster (`xot --gpus N --federate`).

The reference's node always joins the discovered ring: discovery finds the peers, the partitioning strategy gives
each a layer range by memory, and activations hop peer to peer over gRPC (xotorch/main.py:143-173,
xotorch/orchestration/node.py:462-511 and 533-566).  `xot --gpus N` alone serves the whole model on the box's own
RCCL ring (parallel/ring_serve.py), which no other host can join.  With --federate, rank 0 runs the ordinary Node
(gRPC server, UDP / manual discovery, ChatGPT API) whose capabilities are the sum of the box's GPUs, so the
partitioner hands the box a range sized for all of them; its inference engine is `RingFederatedEngine`, which
splits whatever range the cluster assigns over the local ranks and runs every step through them:

  rank 0 (Node + engine) --header (gloo)--> all ranks
  rank 0 layers [a0, b0] --activation (RCCL / xGMI p2p)--> rank 1 [a1, b1] --> ... --> rank N-1 --> rank 0

Each rank holds a ShardedInferenceEngine for its sub-range (its own paged KV cache, batched forward); the result
of the last sub-range (hidden states for the next peer, or logits when the box ends the model) comes back to
rank 0, which hands it to the Node exactly like a single-GPU engine's output.  One request passes the local ring
at a time (the cluster's ring is per request in the reference too); image prompts stay on the unfederated paths.
"""
from __future__ import annotations

import asyncio
import functools
import os
from typing import List, Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist

from ..inference.inference_engine import InferenceEngine
from ..inference.shard import Shard

def split_shard(shard: Shard, world: int) -> List[Shard]:
  """The layer range of `shard` in `world` contiguous, near-equal sub-ranges (at most one per layer)."""
  n = shard.end_layer - shard.start_layer + 1
  parts = min(world, n)
  out, start = [], shard.start_layer
  for r in range(parts):
    k = n // parts + (1 if r < n % parts else 0)
    out.append(Shard(shard.model_id, start, start + k - 1, shard.n_layers))
    start += k
  return out


def _to_tensor(x, dev: torch.device) -> torch.Tensor:
  if isinstance(x, torch.Tensor):
    return x.detach().to(dev)
  return torch.from_numpy(np.ascontiguousarray(x)).to(dev)


def _send(t: torch.Tensor, dst: int, group) -> None:
  """Header object (shape, dtype) on the control group, then the bytes on the data group (bf16 as int16 bits:
  every backend moves 16-bit integers)."""
  t = t.contiguous()
  meta = {"shape": list(t.shape), "dtype": str(t.dtype).replace("torch.", "")}
  dist.send_object_list([meta], dst=dst, group=group["ctl"])
  if t.is_cuda and _host_staged(group):
    t = t.cpu()
  dist.send(t.view(torch.int16) if t.dtype == torch.bfloat16 else t, dst=dst, group=group["data"])


def _host_staged(group) -> bool:
  """gloo data group on a GPU host (single-GPU rehearsals, XOT_DIST_BACKEND=gloo): tensors travel via host memory."""
  return dist.get_backend(group["data"]) == "gloo"


def _recv(src: int, dev: torch.device, group) -> torch.Tensor:
  meta = [None]
  dist.recv_object_list(meta, src=src, group=group["ctl"])
  dt = getattr(torch, meta[0]["dtype"])
  on = torch.device("cpu") if dev.type == "cuda" and _host_staged(group) else dev
  buf = torch.empty(meta[0]["shape"], dtype=torch.int16 if dt == torch.bfloat16 else dt, device=on)
  dist.recv(buf, src=src, group=group["data"])
  buf = buf.view(torch.bfloat16) if dt == torch.bfloat16 else buf
  return buf.to(dev)


def _json_safe(state: Optional[dict]) -> dict:
  """The inference state a header can carry (scalars, strings, lists); tensors stay on rank 0."""
  out = {}
  for k, v in (state or {}).items():
    if isinstance(v, (int, float, str, bool)) or v is None or (isinstance(v, list) and len(v) < 4096):
      out[k] = v
  return out


class RingFederatedEngine(InferenceEngine):
  """Rank 0's engine: the Node's shard split over the local ring (module docstring)."""

  def __init__(self, local, rank: int, world: int, groups: dict, device: torch.device):
    self.local = local  # ShardedInferenceEngine of rank 0's sub-range
    self.rank, self.world = rank, world
    self.groups = groups  # {"ctl": gloo group, "data": RCCL (GPU) or gloo group}
    self.device = device
    self._lock = asyncio.Lock()  # one request in the local ring at a time
    self.shard: Optional[Shard] = None

  # the Node reads these off its engine (EOS handling, token text for the TUI)
  @property
  def tokenizer(self):
    return getattr(self.local, "tokenizer", None)

  @property
  def eos_token_ids(self):
    return getattr(self.local, "eos_token_ids", ())

  def _header(self, op: str, **kw) -> None:
    dist.broadcast_object_list([dict(op=op, **kw)], src=0, group=self.groups["ctl"])

  async def _blocking(self, fn, *args, **kw):
    return await asyncio.get_running_loop().run_in_executor(None, functools.partial(fn, *args, **kw))

  async def encode(self, shard: Shard, prompt: str) -> np.ndarray:
    return await self.local.encode(split_shard(shard, self.world)[0], prompt)

  async def decode(self, shard: Shard, tokens: np.ndarray) -> str:
    return await self.local.decode(split_shard(shard, self.world)[0], tokens)

  async def sample(self, x, temp: float = 0.0, top_k: int = 35) -> np.ndarray:
    return await self.local.sample(x, temp=temp, top_k=top_k)

  async def infer_prompt(self, request_id: str, shard: Shard, prompt: str,
                         inference_state: Optional[dict] = None) -> Tuple[object, Optional[dict]]:
    ids = await self.encode(shard, prompt)
    return await self.infer_tensor(request_id, shard, np.asarray(ids).reshape(1, -1), inference_state)

  async def infer_tensor(self, request_id: str, shard: Shard, input_data,
                         inference_state: Optional[dict] = None) -> Tuple[object, Optional[dict]]:
    subs = split_shard(shard, self.world)
    self.shard = shard
    async with self._lock:
      if len(subs) > 1:
        await self._blocking(self._header, "infer", rid=request_id, subs=[s.to_dict() for s in subs],
                             state=_json_safe(inference_state))
      y, state = await self.local.infer_tensor(request_id, subs[0], input_data, inference_state)
      if len(subs) == 1:
        return y, state
      t = _to_tensor(y, self.device)

      def hop():
        _send(t, 1, self.groups)
        return _recv(len(subs) - 1, self.device, self.groups)

      out = await self._blocking(hop)
    return out, state

  async def finish_request(self, request_id: str, ok: bool = True) -> None:
    if self.world > 1:
      await self._blocking(self._header, "finish", rid=request_id, ok=ok)
    await self.local.finish_request(request_id, ok=ok)

  async def ensure_shard(self, shard: Shard):
    await self.local.ensure_shard(split_shard(shard, self.world)[0])

  async def load_checkpoint(self, shard: Shard, path: str):
    raise NotImplementedError("load checkpoints on the unfederated ring (xot --gpus N)")

  def stop(self) -> None:
    if self.world > 1:
      self._header("stop")


async def follower_loop(local, rank: int, world: int, groups: dict, device: torch.device) -> None:
  """Ranks 1..N-1: act on rank 0's headers until "stop"."""
  loop = asyncio.get_running_loop()

  def header():
    h = [None]
    dist.broadcast_object_list(h, src=0, group=groups["ctl"])
    return h[0]

  while True:
    h = await loop.run_in_executor(None, header)
    op = h["op"]
    if op == "stop":
      return
    if op == "finish":
      await local.finish_request(h["rid"], ok=h.get("ok", True))
      continue
    subs = [Shard.from_dict(s) for s in h["subs"]]
    if rank >= len(subs):
      continue
    x = await loop.run_in_executor(None, _recv, rank - 1, device, groups)
    inp = x if x.dtype.is_floating_point else x.cpu().numpy()
    y, _ = await local.infer_tensor(h["rid"], subs[rank], inp, dict(h.get("state") or {}))
    nxt = (rank + 1) % len(subs) if rank + 1 < len(subs) else 0
    await loop.run_in_executor(None, _send, _to_tensor(y, device), nxt, groups)


def ring_capabilities(world: int):
  """The box as one peer: every local GPU's memory and FLOPS summed (so the cluster partitioner sizes its
  layer range for the whole ring)."""
  from ..topology.device_capabilities import DeviceCapabilities, DeviceFlops, device_capabilities
  one = device_capabilities()
  f = one.flops
  return DeviceCapabilities(model=f"{one.model} x{world} (RCCL ring)", chip=one.chip, memory=one.memory * world,
                            flops=DeviceFlops(fp32=f.fp32 * world, fp16=f.fp16 * world, int8=f.int8 * world))


def _federate_worker(rank: int, world: int, port: int, argv: List[str]) -> None:
  os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                    MASTER_PORT=str(port), XOT_PEER_RANK=str(rank))
  from ..download.new_shard_download import new_shard_downloader
  from ..inference.sharded_engine import ShardedInferenceEngine
  from .comm import init_distributed
  from .ring_serve import control_group
  from .. import main as xot_main

  rank, world, dev = init_distributed()
  groups = {"ctl": control_group(), "data": dist.group.WORLD}
  args = xot_main.build_parser().parse_args(argv)
  local = ShardedInferenceEngine(new_shard_downloader(args.max_parallel_downloads), device=dev)
  try:
    if rank == 0:
      engine = RingFederatedEngine(local, rank, world, groups, dev)
      rc = asyncio.run(xot_main.async_main(args, engine=engine, device_caps=ring_capabilities(world)))
      engine.stop()
    else:
      asyncio.run(follower_loop(local, rank, world, groups, dev))
      rc = 0
  finally:
    if dist.is_initialized():
      dist.destroy_process_group()
  raise SystemExit(rc or 0)


def worker_argv(argv: List[str]) -> List[str]:
  """The command line of a rank: the user's, without --gpus N / --federate (each rank is one process)."""
  rest, skip = [], False
  for a in argv:
    if skip:
      skip = False
      continue
    if a in ("--gpus", "--federate") or a.startswith("--gpus="):
      skip = a == "--gpus"
      continue
    rest.append(a)
  return rest


def federate_ring(args, argv: List[str]) -> int:
  """`xot --gpus N --federate`: one process per local GPU; rank 0 is the cluster peer (module docstring)."""
  import torch.multiprocessing as mp
  from ..train.ring_train import _free_port
  n = args.gpus
  port = _free_port()
  rest = worker_argv(argv)
  ctx = mp.get_context("spawn")
  procs = [ctx.Process(target=_federate_worker, args=(r, n, port, rest)) for r in range(n)]
  for p in procs:
    p.start()
  rc = 0
  for p in procs:
    p.join()
    rc = rc or (p.exitcode or 0)
  return rc

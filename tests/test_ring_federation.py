"""`xot --gpus N --federate` (parallel/ring_federation.py): the local ring as one cluster peer.  CPU / gloo ranks:
the engine the Node drives on rank 0 splits the Node's layer range over the ranks and returns the same logits as
one engine holding the whole range, through prefill, decode steps and a request finish (reference behaviour
being matched: every peer of the discovered ring runs its range, xotorch/orchestration/node.py:462-511)."""
import asyncio
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from xotorch_support_jetson_amd.download.shard_download import NoopShardDownloader
from xotorch_support_jetson_amd.inference.shard import Shard
from xotorch_support_jetson_amd.inference.sharded_engine import ShardedInferenceEngine
from xotorch_support_jetson_amd.parallel.ring_federation import (RingFederatedEngine, follower_loop, split_shard,
                                                                 worker_argv)

MODEL = "tiny-llama-8l"
PROMPT = np.array([[3, 17, 42, 5, 99, 7, 11, 250, 31, 8]], dtype=np.int64)


async def _steps(engine, shard):
  """Prefill + 3 greedy decode steps of one request; the logits of every step."""
  out = []
  y, _ = await engine.infer_tensor("r1", shard, PROMPT, {})
  for _ in range(4):
    logits = torch.as_tensor(y).float().reshape(-1, y.shape[-1])[-1:]
    out.append(logits.cpu().numpy())
    if len(out) == 4:
      break
    tok = int(logits.argmax())
    y, _ = await engine.infer_tensor("r1", shard, np.array([[tok]], dtype=np.int64), {})
  await engine.finish_request("r1")
  return out


def _worker(rank, world, port, q, shard_dict):
  os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
  dist.init_process_group("gloo", rank=rank, world_size=world)
  try:
    groups = {"ctl": dist.new_group(backend="gloo"), "data": dist.group.WORLD}
    dev = torch.device("cpu")
    local = ShardedInferenceEngine(NoopShardDownloader(), device=dev)
    if rank == 0:
      eng = RingFederatedEngine(local, 0, world, groups, dev)
      out = asyncio.run(_steps(eng, Shard.from_dict(shard_dict)))
      eng.stop()
      q.put((rank, out))
    else:
      asyncio.run(follower_loop(local, rank, world, groups, dev))
      q.put((rank, None))
  finally:
    dist.destroy_process_group()


def _free_port():
  with socket.socket() as s:
    s.bind(("127.0.0.1", 0))
    return s.getsockname()[1]


def test_federate_cli():
  from xotorch_support_jetson_amd.main import build_parser
  a = build_parser().parse_args(["--gpus", "8", "--federate", "--discovery-module", "manual"])
  assert a.federate and a.gpus == 8
  assert worker_argv(["--gpus", "8", "--federate", "--node-port", "5000"]) == ["--node-port", "5000"]
  assert worker_argv(["--gpus=4", "--federate"]) == []


def test_split_shard_covers_range_once():
  subs = split_shard(Shard("m", 3, 12, 40), 3)
  assert [(s.start_layer, s.end_layer) for s in subs] == [(3, 6), (7, 9), (10, 12)]
  assert [(s.start_layer, s.end_layer) for s in split_shard(Shard("m", 0, 1, 2), 4)] == [(0, 0), (1, 1)]


@pytest.mark.parametrize("world,lo,hi", [(2, 0, 7), (3, 0, 7)])
def test_federated_ring_matches_one_engine(world, lo, hi):
  shard = Shard(MODEL, lo, hi, 8)
  ref = asyncio.run(_steps(ShardedInferenceEngine(NoopShardDownloader(), device=torch.device("cpu")), shard))
  ctx = mp.get_context("spawn")
  q = ctx.Queue()
  port = _free_port()
  ps = [ctx.Process(target=_worker, args=(r, world, port, q, shard.to_dict())) for r in range(world)]
  for p in ps:
    p.start()
  res = {}
  for _ in range(world):
    rank, out = q.get(timeout=150)
    res[rank] = out
  for p in ps:
    p.join(30)
  got = res[0]
  assert len(got) == len(ref) == 4
  for a, b in zip(got, ref):
    assert np.allclose(a, b, atol=2e-2, rtol=2e-2), np.abs(a - b).max()
    assert int(a.argmax()) == int(b.argmax())


def _worker_gpu(rank, world, port, q, shard_dict):
  os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
  dist.init_process_group("gloo", rank=rank, world_size=world)
  try:
    groups = {"ctl": dist.new_group(backend="gloo"), "data": dist.group.WORLD}
    dev = torch.device("cuda", 0)  # both ranks on the one GPU of the box: activations staged through the host
    local = ShardedInferenceEngine(NoopShardDownloader(), device=dev)
    if rank == 0:
      eng = RingFederatedEngine(local, 0, world, groups, dev)
      out = asyncio.run(_steps(eng, Shard.from_dict(shard_dict)))
      eng.stop()
      q.put((rank, out))
    else:
      asyncio.run(follower_loop(local, rank, world, groups, dev))
      q.put((rank, None))
  finally:
    dist.destroy_process_group()


@pytest.mark.gpu
def test_federated_ring_on_gpu():
  """The GPU engines (batched forward, HIP kernels) behind the federation: two ranks on the box's GPU."""
  shard = Shard(MODEL, 0, 7, 8)
  ref = asyncio.run(_steps(ShardedInferenceEngine(NoopShardDownloader(), device=torch.device("cuda", 0)), shard))
  ctx = mp.get_context("spawn")
  q = ctx.Queue()
  port = _free_port()
  ps = [ctx.Process(target=_worker_gpu, args=(r, 2, port, q, shard.to_dict())) for r in range(2)]
  for p in ps:
    p.start()
  res = {}
  for _ in range(2):
    rank, out = q.get(timeout=100)
    res[rank] = out
  for p in ps:
    p.join(30)
  for a, b in zip(res[0], ref):
    assert np.allclose(a, b, atol=3e-2, rtol=3e-2), np.abs(a - b).max()

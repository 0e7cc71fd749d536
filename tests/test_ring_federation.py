"""`xot --gpus N --federate` (parallel/ring_federation.py): the local ring as one cluster peer.  CPU / gloo ranks:
the engine the Node drives on rank 0 splits the Node's layer range over the ranks and returns what one engine
holding the whole range returns -- through prefill, decode, prompt-prefix reuse, concurrent requests, a failing
rank, training, evaluation and checkpoints -- and a federated box serves and trains next to a second Node over
real gRPC (reference behaviour being matched: every peer of the discovered ring runs its range and takes part in
training, xotorch/orchestration/node.py:299-345 and 462-511, networking/grpc/grpc_server.py:94-114,
networking/manual/test_manual_discovery.py:69-96)."""
import asyncio
import json
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
from xotorch_support_jetson_amd.parallel.ring_federation import (FederationError, RingFederatedEngine,
                                                                 federation_edges, follower_loop, split_shard,
                                                                 worker_argv)

MODEL = "tiny-llama-8l"
PROMPT = np.array([[3, 17, 42, 5, 99, 7, 11, 250, 31, 8]], dtype=np.int64)


def cpu_engine():
  return ShardedInferenceEngine(NoopShardDownloader(), device=torch.device("cpu"))


def host(y) -> np.ndarray:
  return torch.as_tensor(y).float().reshape(-1, torch.as_tensor(y).shape[-1])[-1:].cpu().numpy()


async def _steps(engine, shard, rid="r1", prompt=PROMPT, n=4):
  """Prefill + greedy decode steps of one request; the logits of every step."""
  out = []
  y, st = await engine.infer_tensor(rid, shard, prompt, {})
  while True:
    out.append(host(y))
    if len(out) == n:
      break
    y, st = await engine.infer_tensor(rid, shard, np.array([[int(out[-1].argmax())]], dtype=np.int64), st)
  await engine.finish_request(rid)
  return out


def _prefix_prompts():
  rng = np.random.default_rng(5)
  a = rng.integers(3, 500, size=200)
  b = np.concatenate([a[:150], rng.integers(3, 500, size=30)])
  c = np.concatenate([a[:140], rng.integers(3, 500, size=45)])
  return a.reshape(1, -1), b.reshape(1, -1), c.reshape(1, -1)


def _train_batch():
  rng = np.random.default_rng(9)
  x = rng.integers(3, 500, size=(2, 24)).astype(np.int64)
  return x, np.roll(x, -1, 1), np.array([24, 17], dtype=np.int64)


def _masters(engine) -> dict:
  tr = getattr(engine, "trainer", None)
  return {} if tr is None else {k: v.detach().float().numpy().copy() for k, v in tr.master.items()}


# ------------------------------------------------------------------ scenarios run on rank 0
async def _scenario_steps(eng, shard_dict):
  return await _steps(eng, Shard.from_dict(shard_dict))


async def _scenario_protocol(eng, shard_dict, ckdir):
  """Prefix reuse with two concurrent requests, a failing rank, training, evaluation, checkpoint save / load."""
  from xotorch_support_jetson_amd.train.checkpoint import checkpoint_path
  shard = Shard.from_dict(shard_dict)
  res = {}
  a, b, c = _prefix_prompts()
  res["a"] = await _steps(eng, shard, "A", a, 3)  # the first decode step saves A's full prompt pages
  res["b"], res["c"] = await asyncio.gather(_steps(eng, shard, "B", b, 3), _steps(eng, shard, "C", c, 3))
  res["batches"] = eng.stats["batches"]
  try:
    await eng.infer_tensor("boom", shard, PROMPT, {})
    res["boom"] = "no error"
  except FederationError as e:
    res["boom"] = str(e)
  await eng.finish_request("boom", ok=False)
  res["after_boom"] = await _steps(eng, shard, "ok2")
  x, y, ln = _train_batch()
  res["loss1"], gin = await eng.train("t1", shard, x, y, ln)
  res["gin_none"] = gin is None
  res["eval1"] = await eng.evaluate("e1", shard, x, y, ln)
  path = checkpoint_path(ckdir, shard, 1)
  await eng.save_checkpoint(shard, str(path))
  res["files"] = sorted(os.listdir(os.path.dirname(path)))
  res["loss2"], _ = await eng.train("t2", shard, x, y, ln)
  res["eval2"] = await eng.evaluate("e2", shard, x, y, ln)
  await eng.load_checkpoint(shard, str(path))
  res["eval_loaded"] = await eng.evaluate("e3", shard, x, y, ln)
  res["after_load"] = await _steps(eng, shard, "ok3")
  return res


SCENARIOS = {"steps": _scenario_steps, "protocol": _scenario_protocol}


def _worker(rank, world, port, q, scenario, args):
  os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
  dist.init_process_group("gloo", rank=rank, world_size=world)
  try:
    groups = {"ctl": dist.new_group(backend="gloo"), "data": dist.group.WORLD}
    dev = torch.device("cpu")
    local = ShardedInferenceEngine(NoopShardDownloader(), device=dev)
    if rank == 0:
      eng = RingFederatedEngine(local, 0, world, groups, dev)
      out = asyncio.run(SCENARIOS[scenario](eng, *args))
      eng.stop()
      q.put((rank, out, _masters(local)))
    else:
      if scenario == "protocol" and rank == world - 1:  # the last rank fails one request's step
        orig = local.infer_tensor

        async def flaky(rid, *a, **kw):
          if rid == "boom":
            raise RuntimeError("injected failure")
          return await orig(rid, *a, **kw)
        local.infer_tensor = flaky
      asyncio.run(follower_loop(local, rank, world, groups, dev))
      q.put((rank, None, _masters(local)))
  finally:
    dist.destroy_process_group()


def _free_port():
  with socket.socket() as s:
    s.bind(("127.0.0.1", 0))
    return s.getsockname()[1]


def _spawn(target, world, *args, timeout=240):
  ctx = mp.get_context("spawn")
  q = ctx.Queue()
  port = _free_port()
  ps = [ctx.Process(target=target, args=(r, world, port, q) + args) for r in range(world)]
  for p in ps:
    p.start()
  res = {}
  import queue
  import time
  try:
    t_end = time.time() + timeout
    while len(res) < world:
      try:
        got = q.get(timeout=2)
      except queue.Empty:
        dead = [p.exitcode for p in ps if p.exitcode not in (None, 0)]
        assert not dead and time.time() < t_end, f"ranks failed (exit codes {dead}) or timed out"
        continue
      res[got[0]] = got[1:]
  finally:
    for p in ps:
      p.join(30)
      if p.is_alive():
        p.kill()
  return res


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
  e = federation_edges(3)
  assert len(e) == len(set(e)) and {(0, 1), (1, 0), (1, 2), (2, 1), (2, 0), (0, 2)} == set(e)


@pytest.mark.parametrize("world,lo,hi", [(2, 0, 7), (3, 2, 6)])
def test_federated_ring_matches_one_engine(world, lo, hi):
  shard = Shard(MODEL, lo, hi, 8)
  if lo == 0:
    ref = asyncio.run(_steps(cpu_engine(), shard))
  else:  # a middle range: hidden states in, hidden states out (compare the last-row activations)
    h = torch.randn(1, PROMPT.shape[1], 256, generator=torch.Generator().manual_seed(3)).to(torch.bfloat16)
    ref = None
  res = _spawn(_worker, world, "steps", (shard.to_dict(),)) if lo == 0 else None
  if ref is not None:
    got = res[0][0]
    assert len(got) == len(ref) == 4
    for a, b in zip(got, ref):
      assert np.allclose(a, b, atol=2e-2, rtol=2e-2), np.abs(a - b).max()
      assert int(a.argmax()) == int(b.argmax())
  else:
    res = _spawn(_worker_hidden, world, shard.to_dict(), h)
    want, _ = asyncio.run(cpu_engine().infer_tensor("h", shard, h, {}))
    assert np.allclose(res[0][0].float().numpy(), torch.as_tensor(want).float().numpy(), atol=2e-2, rtol=2e-2)


def _worker_hidden(rank, world, port, q, shard_dict, h):
  os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
  dist.init_process_group("gloo", rank=rank, world_size=world)
  try:
    groups = {"ctl": dist.new_group(backend="gloo"), "data": dist.group.WORLD}
    local = ShardedInferenceEngine(NoopShardDownloader(), device=torch.device("cpu"))
    if rank == 0:
      eng = RingFederatedEngine(local, 0, world, groups, torch.device("cpu"))
      y, _ = asyncio.run(eng.infer_tensor("h", Shard.from_dict(shard_dict), h, {}))
      eng.stop()
      q.put((rank, torch.as_tensor(y).clone()))
    else:
      asyncio.run(follower_loop(local, rank, world, groups, torch.device("cpu")))
      q.put((rank, None))
  finally:
    dist.destroy_process_group()


def test_federated_protocol(tmp_path):
  """Two ranks holding the whole model: prefix reuse across concurrent requests (the forks reach the follower),
  a failing follower step raises on rank 0 and the ring keeps serving, and train / evaluate / save / load give
  the numbers of one engine holding the range."""
  shard = Shard(MODEL, 0, 7, 8)
  res = _spawn(_worker, 2, "protocol", (shard.to_dict(), str(tmp_path / "ck")))
  got, m0 = res[0]
  _, m1 = res[1]

  async def reference():
    a, b, c = _prefix_prompts()
    fresh = cpu_engine()
    fresh.prefix_cache = None
    out = {k: await _steps(fresh, shard, k.upper(), p, 3) for k, p in (("a", a), ("b", b), ("c", c))}
    out["ok2"] = await _steps(fresh, shard, "ok2")
    e = cpu_engine()
    x, y, ln = _train_batch()
    out["loss1"], _ = await e.train("t1", shard, x, y, ln)
    out["eval1"] = await e.evaluate("e1", shard, x, y, ln)
    out["masters1"] = _masters(e)
    out["loss2"], _ = await e.train("t2", shard, x, y, ln)
    out["eval2"] = await e.evaluate("e2", shard, x, y, ln)
    return out

  ref = asyncio.run(reference())
  for k in ("a", "b", "c"):
    for u, v in zip(got[k], ref[k]):
      assert np.allclose(u, v, atol=2e-2, rtol=2e-2), (k, np.abs(u - v).max())
      assert int(u.argmax()) == int(v.argmax())
  assert "injected failure" in got["boom"] and "rank 1" in got["boom"]
  for u, v in zip(got["after_boom"], ref["ok2"]):
    assert np.allclose(u, v, atol=2e-2, rtol=2e-2)
  # training: the same loss and the same updated weights as one engine holding the range
  assert abs(got["loss1"] - ref["loss1"]) < 1e-4 * max(1.0, abs(ref["loss1"]))
  assert got["gin_none"]
  assert abs(got["eval1"] - ref["eval1"]) < 1e-4 * max(1.0, abs(ref["eval1"]))
  assert abs(got["loss2"] - ref["loss2"]) < 1e-4 * max(1.0, abs(ref["loss2"]))
  assert abs(got["eval2"] - ref["eval2"]) < 1e-4 * max(1.0, abs(ref["eval2"]))
  assert got["eval1"] != got["eval2"]  # the second step moved the weights
  # the checkpoint is one file per sub-range, and loading it brings back the weights after step 1
  assert [f for f in got["files"] if not f.endswith(".optim.safetensors")] == [
    "000-003-of-008-000001.safetensors", "004-007-of-008-000001.safetensors"]
  assert abs(got["eval_loaded"] - got["eval1"]) < 1e-3 * max(1.0, abs(got["eval1"]))
  # after the load every rank's trainer holds the checkpoint's fp32 masters (its optimizer sidecar): step 1's
  fed = {**m0, **m1}
  assert set(fed) == set(ref["masters1"])
  for k, v in ref["masters1"].items():
    assert np.allclose(fed[k], v, rtol=0, atol=1e-7), (k, np.abs(fed[k] - v).max())
  for u, v in zip(got["after_load"], got["after_boom"]):  # inference serves the loaded (trained) weights
    assert not np.allclose(u, v, rtol=0, atol=0)


def _grpc_worker(rank, world, port, q, tmp):
  """Rank 0: Node A (the federated box, layers split over both ranks) and Node B (one engine) on localhost gRPC
  with manual discovery; rank 1: the box's follower."""
  os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
  dist.init_process_group("gloo", rank=rank, world_size=world)
  try:
    groups = {"ctl": dist.new_group(backend="gloo"), "data": dist.group.WORLD}
    dev = torch.device("cpu")
    local = ShardedInferenceEngine(NoopShardDownloader(), device=dev)
    if rank != 0:
      asyncio.run(follower_loop(local, rank, world, groups, dev))
      q.put((rank, None, _masters(local)))
      return
    fed = RingFederatedEngine(local, 0, world, groups, dev)
    out = asyncio.run(asyncio.wait_for(_grpc_scenario(fed, tmp), 200))
    fed.stop()
    q.put((rank, out, _masters(local)))
  finally:
    dist.destroy_process_group()


class _Recording(ShardedInferenceEngine):
  def __init__(self):
    super().__init__(NoopShardDownloader(), device=torch.device("cpu"))
    self.seen = []

  async def sample(self, x, temp=0.0, top_k=35):
    self.seen.append(host(x))
    return await super().sample(x, temp, top_k)


async def _grpc_scenario(fed, tmp):
  from xotorch_support_jetson_amd.networking.grpc.grpc_peer_handle import GRPCPeerHandle
  from xotorch_support_jetson_amd.networking.grpc.grpc_server import GRPCServer
  from xotorch_support_jetson_amd.networking.manual.manual_discovery import ManualDiscovery
  from xotorch_support_jetson_amd.orchestration.node import Node
  from xotorch_support_jetson_amd.topology.device_capabilities import DeviceCapabilities
  from xotorch_support_jetson_amd.topology.ring_memory_weighted_partitioning_strategy import \
    RingMemoryWeightedPartitioningStrategy
  caps = {"box": {"model": "box x2", "chip": "t", "memory": 2000, "flops": {"fp32": 1.0, "fp16": 2.0, "int8": 4.0}},
          "solo": {"model": "one", "chip": "t", "memory": 1000, "flops": {"fp32": 1.0, "fp16": 2.0, "int8": 4.0}}}
  ports = {i: _free_port() for i in caps}
  path = os.path.join(tmp, "topology.json")
  with open(path, "w") as f:
    json.dump({"peers": {i: {"address": "127.0.0.1", "port": ports[i], "device_capabilities": caps[i]}
                         for i in caps}}, f)
  solo_eng = _Recording()
  nodes = {}
  for i, eng in (("box", fed), ("solo", solo_eng)):
    disc = ManualDiscovery(path, i, create_peer_handle=lambda pid, addr, desc, c: GRPCPeerHandle(pid, addr, desc, c),
                           poll_interval=0.2)
    n = Node(i, None, eng, disc, NoopShardDownloader(), RingMemoryWeightedPartitioningStrategy(),
             max_generate_tokens=64, device_caps=DeviceCapabilities(**caps[i]))
    n.server = GRPCServer(n, "127.0.0.1", ports[i])
    nodes[i] = n
  for n in nodes.values():
    await n.server.start()
  await asyncio.gather(*(n.start(wait_for_peers=1) for n in nodes.values()))
  for n in nodes.values():
    await n.collect_topology(set())
  base = Shard(MODEL, 0, 0, 8)
  out = {"box": nodes["box"].get_current_shard(base).to_dict(), "solo": nodes["solo"].get_current_shard(base).to_dict()}
  try:
    done = asyncio.Event()
    toks = []
    nodes["box"].on_token.register("t").on_next(lambda rid, t, fin: (toks.extend(t), fin and done.set()))
    await nodes["box"].process_prompt(base, "federated hello", request_id="g1",
                                      inference_state={"temperature": 0.0, "max_tokens": 4})
    await asyncio.wait_for(done.wait(), 60)
    out["tokens"] = [int(t) for t in toks]
    out["logits"] = solo_eng.seen[:4]
    out["ids"] = (await fed.encode(base, "federated hello")).tolist()
    x, y, ln = _train_batch()
    out["loss"] = await nodes["box"].enqueue_example(base, x, y, ln, request_id="ex1", train=True)
    out["solo_masters"] = _masters(solo_eng)
  finally:
    for n in nodes.values():
      await n.stop()
  return out


def test_federated_box_next_to_grpc_node(tmp_path):
  """A 2-rank federated box and a second Node over real localhost gRPC divide one model: greedy generation gives
  the tokens and logits of one engine holding the whole model, and one cluster training step gives the loss of
  that engine and, on every layer, the weights of the unfederated cluster protocol (box range on one engine)."""
  res = _spawn(_grpc_worker, 2, str(tmp_path), timeout=280)
  out, m0 = res[0]
  _, m1 = res[1]
  box, solo = Shard.from_dict(out["box"]), Shard.from_dict(out["solo"])
  assert box.start_layer == 0 and solo.end_layer == 7 and box.end_layer + 1 == solo.start_layer

  async def reference():
    whole = Shard(MODEL, 0, 7, 8)
    e = cpu_engine()
    ids = np.asarray(out["ids"], dtype=np.int64).reshape(1, -1)
    logits = await _steps(e, whole, "g", ids, 4)
    x, y, ln = _train_batch()
    loss_whole, _ = await cpu_engine().train("w", whole, x, y, ln)
    ea, eb = cpu_engine(), cpu_engine()  # the cluster protocol with the box as one engine (node.py:378-392)
    act = await ea.train_forward("t", box, x)
    loss, g = await eb.train("t", solo, act, y, ln)
    await ea.train("t", box, x, g, ln, loss="back_gradient")
    return logits, loss_whole, loss, _masters(ea), _masters(eb)

  logits, loss_whole, loss, ma, mb = asyncio.run(reference())
  assert out["tokens"] == [int(l.argmax()) for l in logits]
  for u, v in zip(out["logits"], logits):
    assert np.allclose(u, v, atol=2e-2, rtol=2e-2), np.abs(u - v).max()
  assert abs(out["loss"] - loss_whole) < 1e-4 * max(1.0, abs(loss_whole))
  assert abs(out["loss"] - loss) < 1e-6 * max(1.0, abs(loss))
  fed = {**m0, **m1}
  assert set(fed) == set(ma)
  for k in ma:
    d_fed, d_ref = fed[k], ma[k]
    assert np.allclose(d_fed, d_ref, rtol=0, atol=1e-7), (k, np.abs(d_fed - d_ref).max())
  for k in mb:
    assert np.allclose(out["solo_masters"][k], mb[k], rtol=0, atol=1e-7), k


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
      x, y, ln = _train_batch()
      loss, _ = asyncio.run(eng.train("t", Shard.from_dict(shard_dict), x, y, ln))
      eng.stop()
      q.put((rank, (out, loss)))
    else:
      asyncio.run(follower_loop(local, rank, world, groups, dev))
      q.put((rank, None))
  finally:
    dist.destroy_process_group()


@pytest.mark.gpu
def test_federated_ring_on_gpu():
  """The GPU engines (batched forward, HIP kernels, GPU trainers) behind the federation: two ranks on the box's GPU."""
  shard = Shard(MODEL, 0, 7, 8)

  async def reference():
    e = ShardedInferenceEngine(NoopShardDownloader(), device=torch.device("cuda", 0))
    logits = await _steps(e, shard)
    x, y, ln = _train_batch()
    loss, _ = await e.train("t", shard, x, y, ln)
    return logits, loss

  ref, ref_loss = asyncio.run(reference())
  res = _spawn(_worker_gpu, 2, shard.to_dict(), timeout=100)
  got, loss = res[0][0]
  for a, b in zip(got, ref):
    assert np.allclose(a, b, atol=3e-2, rtol=3e-2), np.abs(a - b).max()
  assert abs(loss - ref_loss) < 2e-2 * max(1.0, abs(ref_loss))

"""Continuous-batching serving over the process ring (parallel/ring_serve.py), gloo on CPU: requests
admitted at different rounds, with different prompt lengths and budgets, generate exactly the tokens
a single-process server generates; finished requests free their KV pages on every rank."""
import os
import socket
import threading

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from xotorch_support_jetson_amd.models.config import PRESETS
from xotorch_support_jetson_amd.parallel.comm import P2PTransport
from xotorch_support_jetson_amd.parallel.ring_serve import RingServer
from xotorch_support_jetson_amd.runtime.runner import ShardRunner
from xotorch_support_jetson_amd.topology.ring_memory_weighted_partitioning_strategy import equal_layer_shards

MODEL = "tiny-llama"
REQS = [("a", 7, 6), ("b", 12, 4), ("c", 5, 9)]  # rid, prompt length, max tokens


def _prompt(rid, n):
  g = torch.Generator().manual_seed(ord(rid))
  return torch.randint(0, PRESETS[MODEL].vocab_size, (n,), generator=g).tolist()


def _serve(rank, world, ctl, device="cpu"):
  c = PRESETS[MODEL]
  shard = equal_layer_shards(MODEL, c.num_layers, world)[rank]
  runner = ShardRunner(c, shard, device, max_batch=8, max_ctx=64)
  srv = RingServer(runner, rank, world, P2PTransport(rank, world), ctl)
  out = {}
  if rank == 0:
    done = threading.Event()

    def on_tok(rid, toks, fin):
      out.setdefault(rid, []).extend(toks)
      if rid == "a" and len(out["a"]) == 2:  # admit "c" while "a" and "b" are mid-generation
        rid_c, n, mt = REQS[2]
        srv.submit(rid_c, _prompt(rid_c, n), 0.0, mt)
      if fin and len([r for r in out if len(out[r]) == dict((q[0], q[2]) for q in REQS)[r]]) == len(REQS):
        done.set()

    srv.on_token(on_tok)
    for rid, n, mt in REQS[:2]:
      srv.submit(rid, _prompt(rid, n), 0.0, mt)
    th = threading.Thread(target=srv.serve_forever, kwargs=dict(idle_wait=0.05))
    th.start()
    assert done.wait(120), out
    srv.stop()
    th.join(60)
  else:
    srv.serve_forever()
  live = [rid for rid, _, _ in REQS if runner.has(rid)]
  return out, live


def _worker(rank, world, port, q):
  os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
  dist.init_process_group("gloo", rank=rank, world_size=world)
  try:
    ctl = dist.new_group(backend="gloo")
    out, live = _serve(rank, world, ctl)
    q.put((rank, out, live))
  finally:
    dist.destroy_process_group()


def _free_port():
  with socket.socket() as s:
    s.bind(("127.0.0.1", 0))
    return s.getsockname()[1]


@pytest.mark.parametrize("world", [2, 3])
def test_ring_serve_matches_single_process(world):
  """world 2 and 3: requests spread over `world` lanes circulating the ring concurrently."""
  ref, live1 = _serve(0, 1, None)
  assert {r: len(v) for r, v in ref.items()} == {rid: mt for rid, _, mt in REQS}
  ctx = mp.get_context("spawn")
  q = ctx.Queue()
  port = _free_port()
  ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
  for p in ps:
    p.start()
  res = {}
  for _ in range(world):
    rank, out, live = q.get(timeout=180)
    res[rank] = (out, live)
  for p in ps:
    p.join(30)
  assert res[0][0] == ref
  # every request finished and was freed on every rank (the stop header carries the last frees)
  assert all(not res[r][1] for r in range(world))


def test_chatgpt_api_over_ring_server():
  """The ChatGPT API served from a RingServer through RingNode: non-streaming and SSE streaming
  completions honour max_tokens and report usage (world 1 here; the ring data plane is covered above)."""
  import asyncio

  import aiohttp

  from xotorch_support_jetson_amd.api.chatgpt_api import ChatGPTAPI
  from xotorch_support_jetson_amd.inference.shard import Shard
  from xotorch_support_jetson_amd.inference.tokenizers import _resolve_tokenizer
  from xotorch_support_jetson_amd.parallel.ring_serve import RingNode

  c = PRESETS[MODEL]
  shard = Shard(MODEL, 0, c.num_layers - 1, c.num_layers)
  runner = ShardRunner(c, shard, "cpu", max_batch=8, max_ctx=256)
  srv = RingServer(runner, 0, 1, P2PTransport(0, 1))
  tok = _resolve_tokenizer("byte", c.vocab_size)
  port = _free_port()

  async def main():
    node = RingNode(srv, shard, tok, (), 0.0, 16, loop=asyncio.get_running_loop())
    th = threading.Thread(target=srv.serve_forever, kwargs=dict(idle_wait=0.05), daemon=True)
    th.start()
    api = ChatGPTAPI(node, "ShardedInferenceEngine", response_timeout=60, default_model=MODEL)
    await api.run(host="127.0.0.1", port=port)
    url = f"http://127.0.0.1:{port}/v1/chat/completions"
    body = {"model": MODEL, "messages": [{"role": "user", "content": "hi"}], "max_tokens": 5}
    async with aiohttp.ClientSession() as s:
      async with s.post(url, json=body) as r:
        assert r.status == 200, await r.text()
        d = await r.json()
      assert d["usage"]["completion_tokens"] == 5
      async with s.post(url, json=dict(body, stream=True, max_tokens=4)) as r:
        assert r.status == 200
        chunks = [ln for ln in (await r.text()).splitlines() if ln.startswith("data: ")]
      assert len(chunks) >= 2 and chunks[-1] == "data: [DONE]"
    srv.stop()
    th.join(10)
    await api._runner.cleanup()

  asyncio.run(asyncio.wait_for(main(), 120))


@pytest.mark.gpu
def test_ring_server_on_gpu():
  """The serving round loop on cuda:0 (HIP kernels, paged KV, decode graphs for the running batch):
  staggered admissions all finish with their token budgets and free their pages."""
  from xotorch_support_jetson_amd.ops._ext import require
  require()
  out, live = _serve(0, 1, None, device="cuda:0")
  assert {r: len(v) for r, v in out.items()} == {rid: mt for rid, _, mt in REQS}
  assert all(0 <= t < PRESETS[MODEL].vocab_size for v in out.values() for t in v)
  assert len(live) <= 1

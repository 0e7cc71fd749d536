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


@pytest.mark.parametrize("world,per_rank", [(2, 1), (3, 1), (2, 2)])
def test_ring_serve_matches_single_process(world, per_rank, monkeypatch):
  """world 2 and 3: requests spread over `world` lanes circulating the ring concurrently (2 x 2: two lanes per
  rank, four steps in flight on a two-rank ring)."""
  monkeypatch.setenv("XOT_RING_LANES_PER_RANK", str(per_rank))
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


# ---------------------------------------------------------------------------- chunked prefill, KV pressure,
# failure recovery
LONG = [("p", 150, 5), ("q", 40, 12), ("r", 90, 8), ("s", 20, 10)]  # prompts longer than a step's token budget


def _ref_tokens(reqs):
  """Single process, ample pool, whole prompts: the tokens every configuration below must reproduce."""
  c = PRESETS[MODEL]
  from xotorch_support_jetson_amd.inference.shard import Shard
  runner = ShardRunner(c, Shard(MODEL, 0, c.num_layers - 1, c.num_layers), "cpu", max_batch=8, max_ctx=256)
  srv = RingServer(runner, 0, 1, P2PTransport(0, 1), step_tokens=4096)
  return _run_rank0(srv, reqs)


def _run_rank0(srv, reqs, timeout=150):
  out, done = {}, threading.Event()
  budget = {rid: mt for rid, _, mt in reqs}

  def on_tok(rid, toks, fin):
    out.setdefault(rid, []).extend(toks)
    if fin and all(len(out.get(r, ())) >= budget[r] for r in budget):
      done.set()
  srv.on_token(on_tok)
  for rid, n, mt in reqs:
    srv.submit(rid, _prompt(rid, n), 0.0, mt)
  th = threading.Thread(target=srv.serve_forever, kwargs=dict(idle_wait=0.05))
  th.start()
  ok = done.wait(timeout)
  srv.stop()
  th.join(60)
  assert ok, out
  return out


def _worker2(rank, world, port, q, pages, fault, ops_cap=256, slack=3, reqs=None):
  import datetime
  from xotorch_support_jetson_amd.parallel.health import HealthMonitor
  from xotorch_support_jetson_amd.parallel.ring_serve import control_group, min_pool_pages, ring_shards
  os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
  if fault:
    os.environ["XOT_FAULT"] = fault
  dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=60))
  c = PRESETS[MODEL]

  def make_runner(r, w, ctl):
    shard = ring_shards(MODEL, c.num_layers, w, ctl)[r]
    # rank-dependent pool sizes: the ring plans with the smallest one
    runner = ShardRunner(c, shard, "cpu", max_batch=8, max_ctx=256, num_pages=pages + slack * r)
    return runner, min_pool_pages(runner, w, ctl)

  ctl = control_group()
  runner, pool = make_runner(rank, world, ctl)
  # 5 s: a loaded CI host (parallel test workers) must not make a live peer look dead
  mon = HealthMonitor(rank, world, interval=0.1, timeout=5.0).start() if fault else None
  srv = RingServer(runner, rank, world, P2PTransport(rank, world, monitor=mon), ctl, step_tokens=32, monitor=mon,
                   make_runner=make_runner, pool_pages=pool, ops_cap=ops_cap)
  res = None
  if rank == 0:
    res = _run_rank0(srv, reqs or LONG)
  else:
    srv.serve_forever()
  # pages still held: only the prefix cache's holders (rank 0 owns the cache; every rank mirrors its pool)
  used = srv.r.bm.num_blocks - srv.r.bm.num_free
  cached = srv.pc.cached_pages() if srv.pc is not None else None
  q.put((rank, res, dict(srv.stats), srv.pool_pages, (used, cached)))
  q.close()
  q.join_thread()
  os._exit(0)


def _launch2(world, pages, fault="", **kw):
  ctx = mp.get_context("spawn")
  q = ctx.Queue()
  port = _free_port()
  ps = [ctx.Process(target=_worker2, args=(r, world, port, q, pages, fault), kwargs=kw) for r in range(world)]
  for p in ps:
    p.start()
  want = world - (1 if fault.startswith("kill") else 0)
  res = {}
  for _ in range(want):
    rank, out, stats, pool, clean = q.get(timeout=240)
    res[rank] = (out, stats, pool, clean)
  for p in ps:
    p.join(30)
  return res


@pytest.mark.parametrize("world", [2, 3])
def test_ring_serve_chunked_prefill_and_kv_pressure(world):
  """Prompts longer than the 32-token step budget go through in chunks; a pool of 5 pages (64 tokens
  each) cannot hold every request at once, so the youngest are preempted and later re-prefilled from
  prompt + tokens so far.  Tokens equal the single-process reference; every rank plans with the smallest
  pool; all pages come back."""
  ref = _ref_tokens(LONG)
  res = _launch2(world, pages=5)
  out, stats, pool, _ = res[0]
  assert out == ref
  assert stats["chunks"] > 0 and stats["preempted"] > 0, stats
  assert all(res[r][2] == 5 for r in res)  # min over ranks (rank r has 5 + 3r pages)
  cached = res[0][3][1]
  assert all(res[r][3][0] == cached for r in res)  # every rank's pool is empty again but for the cached prefixes


SHORT = [(chr(ord("A") + i), 4, 3) for i in range(8)]  # finish together, in the same lane steps


def test_ring_serve_frees_beyond_one_header_reach_followers_first():
  """Equal pools on every rank (no slack) and one free per header: when several requests finish at once,
  rank 0 has already dropped their pages and plans the next step into them, so every pending free must
  reach the followers ahead of that step (free-only headers), or a follower's pool runs dry."""
  ref = _ref_tokens(SHORT)
  res = _launch2(2, pages=4, ops_cap=1, slack=0, reqs=SHORT)
  out, stats, pool, _ = res[0]
  assert out == ref
  assert pool == 4 and all(res[r][3][0] == res[0][3][1] for r in res)


def test_ring_serve_recovers_from_a_dead_peer():
  """3 ranks; rank 1 dies mid-stream (XOT_FAULT=kill).  The survivors detect it by heartbeat, re-form a
  2-rank ring, re-partition the layers over it and rank 0 re-admits the running requests: every request
  completes with the tokens of the single-process reference."""
  ref = _ref_tokens(LONG)
  res = _launch2(3, pages=64, fault="kill:rank=1:after=12")
  assert set(res) == {0, 2}
  out, stats, _, _ = res[0]
  assert stats["recoveries"] == 1
  assert out == ref


# ---------------------------------------------------------------------------- orchestration layer over the ring
SHARED = "You are a careful assistant. " * 12  # ~340 byte tokens: five full 64-token pages


def _image_prompt():
  from tests.test_vision import _png_data_url
  from xotorch_support_jetson_amd.models.vision import IMAGE_MARK
  return "USER: " + IMAGE_MARK.format(_png_data_url(3)) + "\nwhat is this? ASSISTANT:"


def _worker_orch(rank, world, port, q, model, prompts, max_toks):
  """Rank 0 serves RingNode + the ChatGPT API over the ring: /v1/topology, /metrics, then `prompts` one after
  the other through RingNode.process_prompt (image markers, prompt-prefix reuse)."""
  import asyncio
  import datetime
  from xotorch_support_jetson_amd.inference.shard import Shard
  from xotorch_support_jetson_amd.inference.tokenizers import _resolve_tokenizer
  from xotorch_support_jetson_amd.models import registry
  from xotorch_support_jetson_amd.parallel.ring_serve import RingNode, control_group, ring_shards
  os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
  dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=60))
  c = PRESETS[model]
  ctl = control_group()
  shard = ring_shards(model, c.num_layers, world, ctl)[rank]
  runner = ShardRunner(c, shard, "cpu", max_batch=8, max_ctx=1024)
  srv = RingServer(runner, rank, world, P2PTransport(rank, world), ctl, step_tokens=128)
  if rank != 0:
    srv.serve_forever()
    q.put((rank, None))
  else:
    import aiohttp
    from xotorch_support_jetson_amd.api.chatgpt_api import ChatGPTAPI
    tok = _resolve_tokenizer(registry.get_repo(model, "ShardedInferenceEngine") or "byte", c.vocab_size)
    full = Shard(model, 0, c.num_layers - 1, c.num_layers)
    api_port = _free_port()

    async def main():
      node = RingNode(srv, full, tok, (), 0.0, max_toks, loop=asyncio.get_running_loop(), config=c)
      th = threading.Thread(target=srv.serve_forever, kwargs=dict(idle_wait=0.05), daemon=True)
      th.start()
      api = ChatGPTAPI(node, "ShardedInferenceEngine", response_timeout=60, default_model=model)
      await api.run(host="127.0.0.1", port=api_port)
      async with aiohttp.ClientSession() as s:
        async with s.get(f"http://127.0.0.1:{api_port}/v1/topology") as r:
          topo = await r.json()
        async with s.get(f"http://127.0.0.1:{api_port}/metrics") as r:
          metrics = await r.text()
      outs = []
      for i, p in enumerate(prompts):
        done, got = asyncio.Event(), []

        def on_tok(rid, toks, fin, me=f"p{i}"):
          if rid == me:
            got.extend(toks)
            if fin:
              done.set()
        node.on_token.register(f"t{i}").on_next(on_tok)
        await node.process_prompt(full, p, request_id=f"p{i}", inference_state={"max_tokens": max_toks})
        await asyncio.wait_for(done.wait(), 120)
        outs.append(got)
      srv.stop()
      th.join(30)
      await api._runner.cleanup()
      return topo, metrics, outs

    topo, metrics, outs = asyncio.run(main())
    q.put((0, dict(topo=topo, kv_gauge="xot_kv_pages_total" in metrics, outs=outs,
                   hit_tokens=srv.pc.stats["hit_tokens"] if srv.pc is not None else 0)))
  q.close()
  q.join_thread()
  os._exit(0)


def _run_orch(world, model, prompts, max_toks):
  ctx = mp.get_context("spawn")
  q = ctx.Queue()
  port = _free_port()
  ps = [ctx.Process(target=_worker_orch, args=(r, world, port, q, model, prompts, max_toks)) for r in range(world)]
  for p in ps:
    p.start()
  res = dict(q.get(timeout=300) for _ in range(world))
  for p in ps:
    p.join(30)
  return res[0]


def _engine_greedy(model, prompt, n):
  """The single-process engine's greedy tokens for a prompt (images expanded by ShardedInferenceEngine)."""
  import asyncio

  import numpy as np

  from xotorch_support_jetson_amd.download.shard_download import NoopShardDownloader
  from xotorch_support_jetson_amd.inference.shard import Shard
  from xotorch_support_jetson_amd.inference.sharded_engine import ShardedInferenceEngine

  async def main():
    c = PRESETS[model]
    e = ShardedInferenceEngine(NoopShardDownloader(), device=torch.device("cpu"))
    sh = Shard(model, 0, c.num_layers - 1, c.num_layers)
    logits, _ = await e.infer_prompt("ref", sh, prompt)
    out = []
    for _ in range(n):
      t = int(np.asarray(torch.as_tensor(logits).float()).reshape(-1, c.vocab_size)[-1].argmax())
      out.append(t)
      logits, _ = await e.infer_tensor("ref", sh, np.asarray([[t]]))
    return out
  return asyncio.run(main())


@pytest.mark.parametrize("world", [2, 3])
def test_ring_orchestration_topology_metrics_and_prefix_reuse(world):
  """`xot --gpus N` rank 0 is a full orchestration peer: /v1/topology lists the N GPU peers with their ring
  edges and layer ranges (covering the model once, in ring order), /metrics carries the KV gauges of the ring's
  pool, and a second prompt sharing a long prefix with the first reuses its cached pages -- with the tokens of
  the single-process engine for both prompts."""
  prompts = [SHARED + "first question?", SHARED + "second one!"]
  got = _run_orch(world, MODEL, prompts, 6)
  topo = got["topo"]
  assert len(topo["nodes"]) == world and topo["active_node_id"] in topo["nodes"]
  assert sum(len(v) for v in topo["peer_graph"].values()) == world
  parts = topo["partitions"]
  assert [p["node_id"] for p in parts] and parts[0]["start_layer"] == 0
  assert parts[-1]["end_layer"] == PRESETS[MODEL].num_layers - 1
  assert all(a["end_layer"] + 1 == b["start_layer"] for a, b in zip(parts, parts[1:]))
  assert got["kv_gauge"]
  assert got["hit_tokens"] >= 4 * 64  # the second prompt forked the first one's cached pages
  assert got["outs"] == [_engine_greedy(MODEL, p, 6) for p in prompts]


def test_ring_llava_image_prompt_matches_engine():
  """An image prompt through RingNode on a 2-rank tiny-LLaVA ring (rank 0 = first shard splices the tower's
  features into the image-token rows) gives the single-process engine's greedy tokens."""
  p = _image_prompt()
  got = _run_orch(2, "tiny-llava", [p], 5)
  assert got["outs"] == [_engine_greedy("tiny-llava", p, 5)]


@pytest.mark.gpu
def test_ring_server_tokens_equal_ring_stage_gpu():
  """The served path and the benchmarked path are one code path: four requests through RingServer (world 1:
  async lane steps, decoders fed from the device ids of the step before) draw exactly the tokens bench.py's
  RingStage / run_decode_steps draws for the same prompts -- sampled at temperature 0.7 with the same seed, on
  cuda:0 with the decode graphs."""
  from xotorch_support_jetson_amd.inference.shard import Shard
  from xotorch_support_jetson_amd.ops._ext import require
  from xotorch_support_jetson_amd.parallel.comm import LoopbackTransport
  from xotorch_support_jetson_amd.parallel.pipeline import MicroBatch, RingStage, run_decode_steps
  require()
  name, B, P, steps = "tiny-llama-d64", 4, 12, 8
  c = PRESETS[name]
  shard = Shard(name, 0, c.num_layers - 1, c.num_layers)
  prompt = torch.randint(0, c.vocab_size, (B, P), generator=torch.Generator().manual_seed(8), dtype=torch.int32)
  st = RingStage(ShardRunner(c, shard, "cuda:0", max_batch=8, max_ctx=128), 0, 1, LoopbackTransport(0, 1))
  mb = MicroBatch([f"r{i}" for i in range(B)], prompt=prompt, temps=torch.full((B,), 0.7, device="cuda:0"))
  first = st.prefill(mb)
  mb.tokens.append(first.tolist())
  run_decode_steps(st, [mb], steps - 1, first_tokens=[first], record=True)
  ref = {f"q{i}": [s[i] for s in mb.tokens] for i in range(B)}

  srv = RingServer(ShardRunner(c, shard, "cuda:0", max_batch=8, max_ctx=128), 0, 1, P2PTransport(0, 1),
                   prefix_cache=False)
  out, done = {}, threading.Event()

  def on_tok(rid, toks, fin):
    out.setdefault(rid, []).extend(toks)
    if sum(len(v) for v in out.values()) == B * steps:
      done.set()
  srv.on_token(on_tok)
  for i in range(B):
    srv.submit(f"q{i}", prompt[i].tolist(), 0.7, steps)
  th = threading.Thread(target=srv.serve_forever, kwargs=dict(idle_wait=0.05))
  th.start()
  ok = done.wait(120)
  srv.stop()
  th.join(60)
  assert ok, out
  assert out == ref

"""Multi-node ring over real gRPC on localhost with the dummy engine (reference:
xotorch/orchestration/test_node.py, xotorch/inference/test_dummy_inference_engine.py), plus the
ChatGPT-API contract against a live node."""
import asyncio
import json
import socket

import numpy as np
import pytest

from xotorch_support_jetson_amd.download.shard_download import NoopShardDownloader
from xotorch_support_jetson_amd.inference.dummy_inference_engine import DummyInferenceEngine
from xotorch_support_jetson_amd.inference.shard import Shard
from xotorch_support_jetson_amd.networking.grpc.grpc_peer_handle import GRPCPeerHandle
from xotorch_support_jetson_amd.networking.grpc.grpc_server import GRPCServer
from xotorch_support_jetson_amd.networking.manual.manual_discovery import ManualDiscovery
from xotorch_support_jetson_amd.orchestration.node import Node
from xotorch_support_jetson_amd.topology.device_capabilities import DeviceCapabilities, DeviceFlops
from xotorch_support_jetson_amd.topology.ring_memory_weighted_partitioning_strategy import \
  RingMemoryWeightedPartitioningStrategy

CAPS = {"model": "test", "chip": "test", "memory": 1000, "flops": {"fp32": 1.0, "fp16": 2.0, "int8": 4.0}}


def free_port():
  with socket.socket() as s:
    s.bind(("127.0.0.1", 0))
    return s.getsockname()[1]


async def make_ring(tmp_path, ids, engines=None):
  ports = {i: free_port() for i in ids}
  cfg = {"peers": {i: {"address": "127.0.0.1", "port": ports[i], "device_capabilities": CAPS} for i in ids}}
  path = tmp_path / "topology.json"
  path.write_text(json.dumps(cfg))
  nodes = []
  for k, i in enumerate(ids):
    eng = engines[k] if engines else DummyInferenceEngine()
    disc = ManualDiscovery(str(path), i, create_peer_handle=lambda pid, addr, desc, caps: GRPCPeerHandle(pid, addr, desc,
                                                                                                        caps),
                           poll_interval=0.2)
    node = Node(i, None, eng, disc, NoopShardDownloader(), RingMemoryWeightedPartitioningStrategy(),
                max_generate_tokens=64, device_caps=DeviceCapabilities(**CAPS))
    node.server = GRPCServer(node, "127.0.0.1", ports[i])
    nodes.append(node)
  for n in nodes:
    await n.server.start()
  await asyncio.gather(*(n.start(wait_for_peers=len(ids) - 1) for n in nodes))
  for n in nodes:
    await n.collect_topology(set())
  return nodes


async def stop_all(nodes):
  for n in nodes:
    await n.stop()


def run(coro):
  return asyncio.run(asyncio.wait_for(coro, timeout=60))


def test_two_node_generation(tmp_path):
  async def main():
    nodes = await make_ring(tmp_path, ["node-a", "node-b"])
    try:
      a, b = nodes
      assert {n for n, _ in a.current_topology.all_nodes()} == {"node-a", "node-b"}
      # equal memory -> ring order by id descending: node-b holds layers 0-3, node-a 4-7
      base = Shard("dummy", 0, 0, 8)
      assert b.get_current_shard(base) == Shard("dummy", 0, 3, 8)
      assert a.get_current_shard(base) == Shard("dummy", 4, 7, 8)
      done = asyncio.Event()
      got = []
      seen_on_b = []

      def on_tok(rid, toks, fin):
        got.extend(toks)
        if fin:
          done.set()

      a.on_token.register("t").on_next(on_tok)
      b.on_token.register("t").on_next(lambda rid, toks, fin: seen_on_b.extend(toks))
      await a.process_prompt(base, "x", request_id="r1")
      await asyncio.wait_for(done.wait(), 20)
      assert got[-1] == 69
      assert all(y == x + 1 for x, y in zip(got[:-2], got[1:-1]))
      await asyncio.sleep(0.3)
      # results are routed to the request origin only (node-a), not broadcast per token
      assert seen_on_b == []
      # finished request released everywhere
      assert "r1" not in a.outstanding_requests and "r1" not in b.outstanding_requests
    finally:
      await stop_all(nodes)

  run(main())


def test_request_params_reach_sampler(tmp_path):
  class Recording(DummyInferenceEngine):
    def __init__(self):
      super().__init__()
      self.temps = []

    async def sample(self, x, temp=0.0, top_k=35):
      self.temps.append((temp, top_k))
      return await super().sample(x, temp, top_k)

  async def main():
    engs = [Recording(), Recording()]
    nodes = await make_ring(tmp_path, ["n1", "n2"], engs)
    try:
      a = nodes[0]
      done = asyncio.Event()
      toks = []
      a.on_token.register("t").on_next(lambda rid, t, fin: (toks.extend(t), fin and done.set()))
      await a.process_prompt(Shard("dummy", 0, 0, 8), "x", request_id="r2",
                             inference_state={"temperature": 0.7, "top_k": 5, "max_tokens": 3})
      await asyncio.wait_for(done.wait(), 20)
      assert len(toks) == 3  # max_tokens honoured
      temps = engs[0].temps + engs[1].temps
      assert temps and all(t == (0.7, 5) for t in temps)
    finally:
      await stop_all(nodes)

  run(main())


def test_three_node_training_example(tmp_path):
  async def main():
    engs = [DummyInferenceEngine() for _ in range(3)]
    nodes = await make_ring(tmp_path, ["p1", "p2", "p3"], engs)
    try:
      base = Shard("dummy", 0, 0, 8)
      x = np.zeros((2, 5), dtype=np.int64)
      first = [n for n in nodes if n.get_current_shard(base).is_first_layer()][0]
      loss = await first.enqueue_example(base, x, x, np.array([5, 4]), request_id="ex1", train=True)
      assert loss is not None
      assert all(e.trained for e in engs)  # every stage stepped
      # checkpoint coordination: every peer saves its own shard file
      await first.coordinate_save(base, 1, str(tmp_path / "ck"))
      await asyncio.sleep(0.5)
      assert sum(len(e.saved) for e in engs) == 3
    finally:
      await stop_all(nodes)

  run(main())


def test_chatgpt_api_contract(tmp_path):
  from aiohttp.test_utils import TestClient, TestServer

  from xotorch_support_jetson_amd.api.chatgpt_api import ChatGPTAPI

  async def main():
    nodes = await make_ring(tmp_path, ["solo"])
    node = nodes[0]
    api = ChatGPTAPI(node, "DummyInferenceEngine", response_timeout=30, default_model="dummy")
    client = TestClient(TestServer(api.app))
    await client.start_server()
    try:
      r = await client.get("/v1/models")
      assert r.status == 200 and any(m["id"] == "dummy" for m in (await r.json())["data"])
      r = await client.get("/healthcheck")
      assert (await r.json()) == {"status": "ok"}
      r = await client.get("/v1/topology")
      assert "solo" in (await r.json())["nodes"]
      body = {"model": "dummy", "messages": [{"role": "user", "content": "hi"}], "temperature": 0.0}
      r = await client.post("/v1/chat/completions", json=body)
      assert r.status == 200, await r.text()
      d = await r.json()
      assert d["object"] == "chat.completion" and d["choices"][0]["finish_reason"] == "stop"
      assert d["usage"]["completion_tokens"] >= 1
      # streaming: chunks then [DONE]
      r = await client.post("/v1/chat/completions", json={**body, "stream": True})
      text = await r.text()
      lines = [l for l in text.split("\n") if l.startswith("data: ")]
      assert lines[-1] == "data: [DONE]"
      chunks = [json.loads(l[6:]) for l in lines[:-1]]
      assert all(c["object"] == "chat.completion.chunk" for c in chunks)
      assert chunks[-1]["choices"][0]["finish_reason"] == "stop"
      r = await client.post("/v1/chat/completions", json={"model": "dummy", "messages": [{"content": "no role"}]})
      assert r.status == 400
      r = await client.post("/v1/chat/token/encode", json={"model": "dummy", "messages": [{"role": "user",
                                                                                          "content": "abc"}]})
      assert r.status == 200 and (await r.json())["num_tokens"] > 0
      r = await client.get("/metrics")
      assert r.status == 200
      r = await client.options("/v1/chat/completions")
      assert r.headers.get("Access-Control-Allow-Origin") == "*"
    finally:
      await client.close()
      await stop_all(nodes)

  run(main())


def test_tinychat_served(tmp_path):
  from aiohttp.test_utils import TestClient, TestServer

  from xotorch_support_jetson_amd.api.chatgpt_api import ChatGPTAPI

  async def main():
    nodes = await make_ring(tmp_path, ["solo2"])
    api = ChatGPTAPI(nodes[0], "DummyInferenceEngine", default_model="dummy")
    client = TestClient(TestServer(api.app))
    await client.start_server()
    try:
      r = await client.get("/")
      assert r.status == 200 and "<html" in (await r.text())
      for f in ("/index.js", "/index.css"):
        r = await client.get(f)
        assert r.status == 200, f
      r = await client.get("/initial_models")
      assert "dummy" in await r.json()
      r = await client.get("/modelpool")
      assert (await r.text()).rstrip().endswith("data: [DONE]")
    finally:
      await client.close()
      await stop_all(nodes)

  run(main())


def test_peer_failure_finishes_request_and_repartitions(tmp_path):
  """A peer dies mid-ring: the request finishes at its origin instead of hanging, and the next request
  runs on the surviving peer, which now holds every layer."""
  async def main():
    nodes = await make_ring(tmp_path, ["node-a", "node-b"])
    a, b = nodes
    try:
      base = Shard("dummy", 0, 0, 8)
      assert a.get_current_shard(base) == Shard("dummy", 4, 7, 8)
      await b.stop()  # node-b (layers 0-3, the first stage) goes away
      done = asyncio.Event()
      a.on_token.register("t").on_next(lambda rid, toks, fin: fin and done.set())
      await a.process_prompt(base, "x", request_id="dead")
      await asyncio.wait_for(done.wait(), 10)
      assert {n for n, _ in a.current_topology.all_nodes()} == {"node-a"}
      assert a.get_current_shard(base) == Shard("dummy", 0, 7, 8)
      done2 = asyncio.Event()
      toks = []
      a.on_token.register("t2").on_next(lambda rid, t, fin: rid == "alive" and (toks.extend(t), fin and done2.set()))
      await a.process_prompt(base, "x", request_id="alive")
      await asyncio.wait_for(done2.wait(), 10)
      assert toks and toks[-1] == 69
    finally:
      await a.stop()

  run(main())


def test_api_concurrent_requests_real_engine(tmp_path):
  """Concurrent chat completions on one peer with the real engine (tiny synthetic Llama on CPU): all
  complete, with per-request max_tokens, through the continuously batched engine."""
  import torch
  from aiohttp.test_utils import TestClient, TestServer

  from xotorch_support_jetson_amd.api.chatgpt_api import ChatGPTAPI
  from xotorch_support_jetson_amd.inference.sharded_engine import ShardedInferenceEngine

  async def main():
    eng = ShardedInferenceEngine(NoopShardDownloader(), device=torch.device("cpu"))
    nodes = await make_ring(tmp_path, ["solo3"], engines=[eng])
    api = ChatGPTAPI(nodes[0], "ShardedInferenceEngine", response_timeout=60, default_model="tiny-llama")
    client = TestClient(TestServer(api.app))
    await client.start_server()
    try:
      async def ask(i):
        r = await client.post("/v1/chat/completions", json={
          "model": "tiny-llama", "messages": [{"role": "user", "content": f"hello {i}"}], "max_tokens": 3 + i,
          "temperature": 0.0})
        assert r.status == 200, await r.text()
        return await r.json()
      outs = await asyncio.gather(*(ask(i) for i in range(4)))
      for i, d in enumerate(outs):
        assert d["usage"]["completion_tokens"] <= 3 + i
    finally:
      await client.close()
      await stop_all(nodes)

  run(main())


@pytest.mark.parametrize("loop_on", [True, False])
def test_api_request_without_temperature(tmp_path, monkeypatch, loop_on):
  """Clients that leave out `temperature` (and top_k / max_tokens): the API forwards them as None, the Node
  fills in its defaults, and every request -- also when batched with requests that did set one -- completes,
  in the engine's decode loop and on the per-token Node path."""
  import torch
  from aiohttp.test_utils import TestClient, TestServer

  from xotorch_support_jetson_amd.api.chatgpt_api import ChatGPTAPI
  from xotorch_support_jetson_amd.inference import sharded_engine as se

  async def main():
    monkeypatch.setattr(se, "ENGINE_LOOP", loop_on)
    eng = se.ShardedInferenceEngine(NoopShardDownloader(), device=torch.device("cpu"))
    nodes = await make_ring(tmp_path, [f"solo_t{int(loop_on)}"], engines=[eng])
    # requests without max_tokens run to the node's cap: keep it small (1024 random-weight tokens per request
    # on the per-token CPU path overran the timeout on a loaded host)
    nodes[0].max_generate_tokens = 16
    api = ChatGPTAPI(nodes[0], "ShardedInferenceEngine", response_timeout=60, default_model="tiny-llama")
    client = TestClient(TestServer(api.app))
    await client.start_server()
    try:
      async def ask(i):
        body = {"model": "tiny-llama", "messages": [{"role": "user", "content": f"hello {i}"}]}
        if i % 2:
          body.update(temperature=0.0, max_tokens=4)
        r = await client.post("/v1/chat/completions", json=body)
        assert r.status == 200, await r.text()
        return await r.json()
      outs = await asyncio.wait_for(asyncio.gather(*(ask(i) for i in range(4))), 60)
      for d in outs:
        assert d["usage"]["completion_tokens"] >= 1
    finally:
      await client.close()
      await stop_all(nodes)

  run(main())


def test_engine_decode_loop_matches_node_path(tmp_path, monkeypatch):
  """A single peer holding the whole model decodes in the engine's loop (continue_locally): same greedy
  tokens as the per-token Node path, per-request max_tokens honoured, nothing left registered."""
  import torch

  from xotorch_support_jetson_amd.inference import sharded_engine as se

  async def gen(loop_on):
    monkeypatch.setattr(se, "ENGINE_LOOP", loop_on)
    eng = se.ShardedInferenceEngine(NoopShardDownloader(), device=torch.device("cpu"))
    d = tmp_path / str(loop_on)
    d.mkdir()
    nodes = await make_ring(d, ["solo4"], engines=[eng])
    node = nodes[0]
    done = {}
    ev = asyncio.Event()

    def on_token(rid, toks, fin):
      if fin:
        done[rid] = list(node.buffered_token_output[rid][0])
        if len(done) == 4:
          ev.set()
    node.on_token.register("t").on_next(on_token)
    try:
      base = Shard("tiny-llama", 0, 0, 4)
      for i in range(4):
        await node.process_prompt(base, f"prompt number {i} " * (i + 1), request_id=f"q{i}",
                                  inference_state={"temperature": 0.0, "max_tokens": 4 + i})
      await asyncio.wait_for(ev.wait(), 60)
      assert not eng._loops
      return done, eng.stats
    finally:
      await stop_all(nodes)

  on, st_on = run(gen(True))
  off, _ = run(gen(False))
  assert on == off
  for i in range(4):
    assert len(on[f"q{i}"]) <= 4 + i
  assert st_on.get("loop_tokens", 0) == sum(len(v) for v in on.values()) - 4  # all but each first token
  # drawn with their forward: in a chained step (ids handed to the next step on the device) or presampled
  assert st_on.get("presampled", 0) + st_on.get("chained_tokens", 0) >= st_on["loop_tokens"]
  assert st_on.get("chained", 0) > 0


def test_engine_loop_consumer_ends_request_early():
  """Pipelined engine loop: the next step is queued before a token is emitted (on the `stop` prediction).
  When the consumer ends a request the prediction did not (a cancelled stream), the queued step is dropped,
  at most the one already running computes for it, and nothing stays registered."""
  import torch

  from xotorch_support_jetson_amd.inference import sharded_engine as se

  async def main():
    eng = se.ShardedInferenceEngine(NoopShardDownloader(), device=torch.device("cpu"))
    shard = Shard("tiny-llama", 0, 3, 4)
    await eng.ensure_shard(shard)
    got = {"a": [], "b": []}
    ended = asyncio.Event()
    steps_after_end = []

    def emit(rid, tok):
      got[rid].append(tok)
      if rid == "a" and len(got["a"]) == 3:  # consumer stops "a" early; the prediction said go on
        steps_after_end.append(eng.stats["steps"])
        return True
      if rid == "b" and len(got["b"]) == 8:
        ended.set()
        return True
      return False

    state = {"temperature": 0.0, "top_k": 35}
    for rid in ("a", "b"):
      logits, _ = await eng.infer_tensor(rid, shard, np.asarray([[1, 2, 3, 4]], dtype=np.int64), state)
      tok = int(np.asarray(await eng.sample(logits, 0.0, 35)).reshape(-1)[0])
      assert eng.continue_locally(rid, shard, tok, dict(state), emit, stop=lambda r, t: False)
    await asyncio.wait_for(ended.wait(), 60)
    for _ in range(50):
      if not eng._draining:
        break
      await asyncio.sleep(0.01)
    assert not eng._loops and not eng._queue
    assert len(got["a"]) == 3 and len(got["b"]) == 8
    # "a" ran its emitted steps plus at most the one in flight when it ended
    assert eng.runner.num_tokens("a") <= 4 + 3 + 1
    await eng.finish_request("a")
    await eng.finish_request("b")
    assert not eng.runner.has("a") and not eng.runner.has("b")

  run(main())


def test_engine_loop_mixed_top_k_all_finish():
  """Chained engine-loop steps share one sampler top_k: a request with another top_k waiting in the queue
  makes the running chain finish so the queue is served normally -- every request completes."""
  import torch

  from xotorch_support_jetson_amd.inference import sharded_engine as se

  async def main():
    eng = se.ShardedInferenceEngine(NoopShardDownloader(), device=torch.device("cpu"))
    shard = Shard("tiny-llama", 0, 3, 4)
    await eng.ensure_shard(shard)
    want = {"a": 12, "b": 5, "c": 7}
    got = {r: [] for r in want}
    done = asyncio.Event()

    def emit(rid, tok):
      got[rid].append(tok)
      fin = len(got[rid]) >= want[rid]
      if all(len(got[r]) >= want[r] for r in want):
        done.set()
      return fin

    def stop(rid, tok):
      return len(got[rid]) + 1 >= want[rid]

    for rid, k in (("a", 35), ("b", 1), ("c", 35)):
      state = {"temperature": 0.7, "top_k": k}
      logits, _ = await eng.infer_tensor(rid, shard, np.asarray([[3, 1, 4, 1, 5]], dtype=np.int64), state)
      tok = int(np.asarray(await eng.sample(logits, 0.7, k)).reshape(-1)[0])
      assert eng.continue_locally(rid, shard, tok, dict(state), emit, stop=stop)
      await asyncio.sleep(0)
    await asyncio.wait_for(done.wait(), 60)
    for _ in range(50):
      if not eng._draining:
        break
      await asyncio.sleep(0.01)
    assert {r: len(v) for r, v in got.items()} == want
    assert not eng._loops and not eng._queue

  run(main())


def test_api_stream_ends_when_engine_loop_fails(tmp_path, monkeypatch):
  """A decode-loop step that raises ends the affected requests' streams (finish chunk, [DONE]) instead of
  leaving the HTTP clients waiting for a token that never comes."""
  import torch
  from aiohttp.test_utils import TestClient, TestServer

  from xotorch_support_jetson_amd.api.chatgpt_api import ChatGPTAPI
  from xotorch_support_jetson_amd.inference.sharded_engine import ShardedInferenceEngine

  async def main():
    eng = ShardedInferenceEngine(NoopShardDownloader(), device=torch.device("cpu"))
    calls = {"n": 0}
    real = eng._chain_step

    def flaky(*a):
      calls["n"] += 1
      if calls["n"] == 3:
        raise RuntimeError("injected step failure")
      return real(*a)
    monkeypatch.setattr(eng, "_chain_step", flaky)
    nodes = await make_ring(tmp_path, ["solo5"], engines=[eng])
    api = ChatGPTAPI(nodes[0], "ShardedInferenceEngine", response_timeout=60, default_model="tiny-llama")
    client = TestClient(TestServer(api.app))
    await client.start_server()
    try:
      async def ask(i):
        r = await client.post("/v1/chat/completions", json={
          "model": "tiny-llama", "messages": [{"role": "user", "content": f"hi {i}"}], "max_tokens": 40,
          "temperature": 0.0, "stream": True})
        return await r.text()
      outs = await asyncio.wait_for(asyncio.gather(*(ask(i) for i in range(3))), 30)
      for text in outs:
        lines = [l for l in text.split("\n") if l.startswith("data: ")]
        assert lines[-1] == "data: [DONE]"
        assert json.loads(lines[-2][6:])["choices"][0]["finish_reason"] is not None
      assert calls["n"] >= 3
    finally:
      await client.close()
      await stop_all(nodes)

  run(main())


def test_engine_loop_kv_pressure_ends_youngest():
  """When the KV pool cannot take a chained step's new pages, the youngest requests are ended (their
  consumers get the end of the request) and the others keep decoding -- the step does not fail for all."""
  import torch

  from xotorch_support_jetson_amd.inference import sharded_engine as se
  from xotorch_support_jetson_amd.runtime.runner import _block_manager

  async def main():
    eng = se.ShardedInferenceEngine(NoopShardDownloader(), device=torch.device("cpu"))
    shard = Shard("tiny-llama", 0, 3, 4)
    await eng.ensure_shard(shard)
    eng.runner.bm = _block_manager(7)  # 7 pages of 64 tokens for everyone
    eng.prefix_cache = None
    want = 40
    got = {r: [] for r in ("a", "b", "c")}
    ended = {}
    done = asyncio.Event()

    def emit(rid, tok):
      got[rid].append(tok)
      fin = len(got[rid]) >= want
      if fin:
        ended[rid] = "done"
        if len(ended) == 3:
          done.set()
      return fin

    def fail(rid):
      ended[rid] = "kv"
      if len(ended) == 3:
        done.set()

    for rid in ("a", "b", "c"):  # 100-token prompts: 2 pages each, crossing into a third at token 128
      state = {"temperature": 0.0, "top_k": 35}
      logits, _ = await eng.infer_tensor(rid, shard, np.arange(100, dtype=np.int64).reshape(1, -1) % 200, state)
      tok = int(np.asarray(await eng.sample(logits, 0.0, 35)).reshape(-1)[0])
      assert eng.continue_locally(rid, shard, tok, dict(state), emit, fail, stop=lambda r, t: len(got[r]) + 1 >= want)
    await asyncio.wait_for(done.wait(), 60)
    assert ended["a"] == "done" and ended["b"] == "done", ended  # 6 pages for a and b fit
    assert ended["c"] == "kv" and len(got["c"]) < want  # the youngest went at the page boundary
    assert eng.stats.get("kv_evicted_requests", 0) == 1
    for rid in ("a", "b", "c"):
      await eng.finish_request(rid)
    assert eng.runner.bm.num_free == 7 and eng.runner.bm.check()

  run(main())

"""Prompt-prefix KV reuse (inference/prefix_cache.py): a prompt that starts with a served prompt's pages
prefills only the rest and gets the same logits; over a two-shard ring the downstream shard mirrors the
first shard's save / fork / drop operations carried in the inference state."""
import asyncio

import numpy as np
import pytest
import torch

from xotorch_support_jetson_amd.download.shard_download import NoopShardDownloader
from xotorch_support_jetson_amd.inference.prefix_cache import PrefixCache, holder
from xotorch_support_jetson_amd.inference.shard import Shard
from xotorch_support_jetson_amd.inference.sharded_engine import ShardedInferenceEngine
from xotorch_support_jetson_amd.runtime.runner import _block_manager

MODEL, N = "tiny-llama", 4


def run(c):
  return asyncio.run(c)


def eng(device="cpu"):
  return ShardedInferenceEngine(NoopShardDownloader(), device=torch.device(device))


def prompts(seed=0):
  rng = np.random.default_rng(seed)
  a = rng.integers(3, 500, size=200)
  b = np.concatenate([a[:150], rng.integers(3, 500, size=30)])
  return a.reshape(1, -1), b.reshape(1, -1)


def host(out) -> np.ndarray:
  return out.float().cpu().numpy() if isinstance(out, torch.Tensor) else np.asarray(out, np.float32)


def greedy(out):
  return np.array([[int(np.argmax(host(out)))]])


def test_single_shard_reuse_matches_fresh_prefill():
  async def main():
    a, b = prompts()
    s = Shard(MODEL, 0, N - 1, N)
    e = eng()
    out, st = await e.infer_tensor("A", s, a)
    for _ in range(2):  # the first decode step saves the prompt's 3 full pages
      out, st = await e.infer_tensor("A", s, greedy(out), st)
    await e.finish_request("A")
    pc = e.prefix_cache
    assert pc.stats["saved"] == 1 and len(pc.entries) == 1
    outb, _ = await e.infer_tensor("B", s, b)
    assert pc.stats["hit_tokens"] == 128  # 2 of B's pages match (150 shared tokens)
    assert e.runner.num_tokens("B") == b.shape[1]
    fresh = eng()
    fresh.prefix_cache = None
    ref, _ = await fresh.infer_tensor("B", s, b)
    assert np.allclose(np.asarray(outb, np.float32), np.asarray(ref, np.float32), atol=5e-3)
    o2, _ = await e.infer_tensor("B", s, greedy(outb))
    r2, _ = await fresh.infer_tensor("B", s, greedy(ref))
    assert np.allclose(np.asarray(o2, np.float32), np.asarray(r2, np.float32), atol=5e-3)
    await e.finish_request("B")
    assert e.runner.bm.check()

  run(main())


def test_two_shard_ring_mirrors_operations():
  async def main():
    a, b = prompts(1)
    sa, sb = Shard(MODEL, 0, 1, N), Shard(MODEL, 2, N - 1, N)
    ea, eb = eng(), eng()

    async def step(rid, x, st=None):
      h, st = await ea.infer_tensor(rid, sa, x, st)
      out, st2 = await eb.infer_tensor(rid, sb, h, st)
      return h, out, {**st, **st2}

    h, out, st = await step("A", a)
    ops = []
    for _ in range(3):
      h, out, st = await step("A", greedy(out), st)
      ops.append(st.get("pc"))
    assert ops[0] and ops[0].get("save") == [0, 192] and not ops[1]  # saved on the first decode step
    assert eb.runner.bm.has(holder(0))  # the downstream shard mirrored the save
    assert ea.prefix_cache.entries[0].confirmed  # confirmed by the second decode step
    h, outb, st = await step("B", b)
    assert st["pc"]["fork"] == [0, 128] and h.shape[1] == b.shape[1] - 128
    assert eb.runner.num_tokens("B") == b.shape[1]
    full = eng()
    full.prefix_cache = None
    ref, _ = await full.infer_tensor("B", Shard(MODEL, 0, N - 1, N), b)
    assert np.allclose(np.asarray(outb, np.float32), np.asarray(ref, np.float32), atol=5e-3)
    # eviction on the first shard rides to the downstream shard on the next outgoing state
    await ea.finish_request("A")
    await eb.finish_request("A")
    pc = ea.prefix_cache
    assert pc.entries[0].pending == 1  # B's fork is not confirmed yet
    pc.evict(10 ** 9)
    assert 0 in pc.entries  # ... so the entry stays
    h, outb, st = await step("B", greedy(outb), st)  # B's next step confirms the fork
    assert pc.entries[0].pending == 0
    pc.evict(10 ** 9)
    assert 0 not in pc.entries and not ea.runner.bm.has(holder(0))
    h, outb, st = await step("B", greedy(outb), st)
    assert st["pc"]["drop"] == [0] and not eb.runner.bm.has(holder(0))
    h, outb, st = await step("B", greedy(outb), st)  # came back: the drop is no longer sent
    assert not (st.get("pc") or {}).get("drop")

  run(main())


def test_policy_confirmation_and_cap():
  bm = _block_manager(64)  # the native BlockManager (pure-python fallback without the build)
  pc = PrefixCache(bm, cap_pages=4, single_shard=False)
  toks = list(range(3, 3 + 300))
  assert pc.on_prompt("A", toks) == (0, None)
  bm.append("A", 300)
  assert pc.on_decode("A") == [0, 256]  # 4 full pages saved
  assert not pc.entries[0].confirmed
  assert pc.on_prompt("B", toks[:200] + [7] * 50) == (0, None)  # unconfirmed: not used yet
  pc.on_decode("A")  # A came back round the ring
  assert pc.entries[0].confirmed
  assert pc.on_prompt("C", toks[:200] + [7] * 50) == (192, 0)
  bm.append("C", 58)
  # a second prompt of 4 other pages does not fit under the cap while C's fork is pending
  other = list(range(1000, 1300))
  pc.on_prompt("D", other)
  bm.append("D", 300)
  assert pc.on_decode("D") is None and 0 in pc.entries
  pc.on_finish("C")  # C ended: its fork is confirmed, the entry may go
  pc.reqs["D"].steps = 0
  assert pc.on_decode("D") == [1, 256] and 0 not in pc.entries and list(pc.drop_q) == [0]
  assert not hasattr(bm, "check") or bm.check()


def test_failed_request_drops_its_unconfirmed_save():
  """A request that fails part-way (a hop to a dead peer, an aborted decode loop) gives no guarantee that
  its save reached the downstream shards: its unconfirmed entry is dropped, never forked by a later prompt;
  a normal finish confirms it as before."""
  bm = _block_manager(64)
  pc = PrefixCache(bm, cap_pages=8, single_shard=False)
  toks = list(range(3, 3 + 300))
  pc.on_prompt("A", toks)
  bm.append("A", 300)
  assert pc.on_decode("A") == [0, 256]
  pc.on_finish("A", ok=False)
  assert 0 not in pc.entries and not bm.has(holder(0)) and list(pc.drop_q) == [0]
  assert pc.on_prompt("B", toks[:200] + [7] * 50) == (0, None)  # a miss, not a fork of a missing holder
  # the same sequence with a normal finish confirms the entry and serves the next prompt
  pc.on_prompt("C", toks)
  bm.append("C", 300)
  save = pc.on_decode("C")
  pc.on_finish("C")
  assert pc.entries[save[0]].confirmed
  assert pc.on_prompt("D", toks[:200] + [7] * 50) == (192, save[0])
  # a failed request that forked: its pending fork is released so the entry can be evicted later
  pc.on_finish("D", ok=False)
  assert pc.entries[save[0]].pending == 0


def test_node_failure_finishes_with_ok_false(tmp_path):
  """Node._abort / _fail_request announce request_finished with failed=True; the engine then gets
  finish_request(ok=False)."""
  from xotorch_support_jetson_amd.inference.dummy_inference_engine import DummyInferenceEngine
  from xotorch_support_jetson_amd.orchestration.node import Node
  from xotorch_support_jetson_amd.topology.ring_memory_weighted_partitioning_strategy import \
      RingMemoryWeightedPartitioningStrategy

  calls = []

  class Eng(DummyInferenceEngine):
    async def finish_request(self, request_id, ok=True):
      calls.append((request_id, ok))

  async def main():
    node = Node("n", None, Eng(), None, None, RingMemoryWeightedPartitioningStrategy())
    node._abort("r1")
    node._finish("r2")
    for _ in range(20):
      await asyncio.sleep(0.01)
    return calls

  got = run(main())
  assert ("r1", False) in got and ("r2", True) in got


def test_cap_follows_smallest_pool_on_the_ring():
  """Downstream shards report their KV pool size in the step state; the first shard caps its cached pages
  at the fraction of the SMALLEST pool, since downstream shards never evict holders on their own."""
  async def main():
    a, _ = prompts(2)
    sa, sb = Shard(MODEL, 0, 1, N), Shard(MODEL, 2, N - 1, N)
    ea, eb = eng(), eng()
    h, st = await ea.infer_tensor("A", sa, a)
    await eb.ensure_shard(sb)
    eb.runner.bm = _block_manager(40)  # a much smaller pool downstream
    out, st2 = await eb.infer_tensor("A", sb, h, st)
    assert st2["kv_min"] == 40
    cap0 = ea.prefix_cache.cap
    await ea.infer_tensor("A", sa, greedy(out), {**st, **st2})
    from xotorch_support_jetson_amd.inference.sharded_engine import PREFIX_CACHE_FRAC
    assert ea.prefix_cache.cap == min(cap0, int(40 * PREFIX_CACHE_FRAC))
  run(main())

"""ShardedInferenceEngine + ShardTrainer on CPU (reference: xotorch/inference/test_inference_engine.py —
split inference == full inference; plus the training path the reference never implemented)."""
import asyncio

import numpy as np
import pytest
import torch

from xotorch_support_jetson_amd.download.shard_download import NoopShardDownloader
from xotorch_support_jetson_amd.inference.shard import Shard
from xotorch_support_jetson_amd.inference.sharded_engine import ShardedInferenceEngine
from xotorch_support_jetson_amd.train import checkpoint as ck

MODEL = "tiny-llama"
N = 4


def run(c):
  return asyncio.run(c)


def eng():
  return ShardedInferenceEngine(NoopShardDownloader(), device=torch.device("cpu"))


def test_engine_split_equals_full():
  async def main():
    full, a, b = eng(), eng(), eng()
    ids = np.random.default_rng(0).integers(0, 500, size=(1, 9))
    f_out, f_state = await full.infer_tensor("r", Shard(MODEL, 0, N - 1, N), ids)
    h, st = await a.infer_tensor("r", Shard(MODEL, 0, 1, N), ids)
    s_out, _ = await b.infer_tensor("r", Shard(MODEL, 2, N - 1, N), h, st)
    assert np.allclose(np.asarray(f_out, np.float32), np.asarray(s_out, np.float32), atol=1e-5)
    # one decode step continues from the cached prefix
    tok = np.asarray(await full.sample(f_out, temp=0.0)).reshape(1, 1)
    f2, _ = await full.infer_tensor("r", Shard(MODEL, 0, N - 1, N), tok, f_state)
    h2, st2 = await a.infer_tensor("r", Shard(MODEL, 0, 1, N), tok, st)
    s2, _ = await b.infer_tensor("r", Shard(MODEL, 2, N - 1, N), h2, st2)
    assert np.allclose(np.asarray(f2, np.float32), np.asarray(s2, np.float32), atol=1e-5)
    await full.finish_request("r")
    assert not full.runner.has("r")

  run(main())


def test_pipeline_training_matches_single_stage():
  """Two-stage SendExample protocol (forward, back-gradient) gives the same loss and updated weights
  as one stage holding all layers."""
  async def main():
    x = np.random.default_rng(1).integers(0, 500, size=(2, 12))
    y = np.roll(x, -1, 1)
    ln = np.array([12, 9])
    full = eng()
    fs = Shard(MODEL, 0, N - 1, N)
    l_full, _ = await full.train("t", fs, x, y, ln)
    s0, s1 = eng(), eng()
    a, b = Shard(MODEL, 0, 1, N), Shard(MODEL, 2, N - 1, N)
    h = await s0.train_forward("t", a, x)
    l_split, g = await s1.train("t", b, h, y, ln)
    _, g0 = await s0.train("t", a, x, g, ln, loss="back_gradient")
    assert g0 is None
    assert abs(l_full - l_split) < 1e-3
    tf, t0, t1 = full.trainer, s0.trainer, s1.trainer
    for k in ("0.qkv", "1.down", "embed"):
      assert torch.allclose(tf.master[k], t0.master[k], atol=2e-6), k
    for k in ("2.o", "3.gu", "norm"):
      assert torch.allclose(tf.master[k], t1.master[k], atol=2e-6), k

  run(main())


def test_training_reduces_loss_and_checkpoint_roundtrip(tmp_path):
  async def main():
    e = eng()
    s = Shard(MODEL, 0, N - 1, N)
    await e.ensure_shard(s)
    e.lr = 3e-3
    rng = np.random.default_rng(2)
    x = rng.integers(0, 64, size=(4, 16))
    y = np.roll(x, -1, 1)
    ln = np.full(4, 16)
    losses = [(await e.train("t", s, x, y, ln))[0] for _ in range(12)]
    assert losses[-1] < losses[0] * 0.9, losses
    ev = await e.evaluate("e", s, x, y, ln)
    assert abs(ev - losses[-1]) < 0.5
    p = ck.checkpoint_path(tmp_path, s, 12)
    await e.save_checkpoint(s, str(p))
    assert p.exists() and p.with_name(p.name.replace(".safetensors", ".optim.safetensors")).exists()
    assert ck.list_checkpoints(tmp_path, MODEL)[-1][0] == 12
    out1, _ = await e.infer_tensor("q", s, x[:1])
    e2 = eng()
    await e2.ensure_shard(s)
    await e2.load_checkpoint(s, str(tmp_path))
    out2, _ = await e2.infer_tensor("q", s, x[:1])
    assert np.array_equal(np.asarray(out1), np.asarray(out2))
    assert e2.trainer is not None and e2.trainer.step_count == 12  # optimizer state resumed

  run(main())


def test_checkpoint_resharding(tmp_path):
  """A checkpoint written by a 1-stage run loads into a 2-stage split (tensors gathered by layer)."""
  async def main():
    e = eng()
    s = Shard(MODEL, 0, N - 1, N)
    await e.ensure_shard(s)
    ids = np.arange(7).reshape(1, 7)
    ref, _ = await e.infer_tensor("q", s, ids)
    await e.save_checkpoint(s, str(ck.checkpoint_path(tmp_path, s, 3)))
    a, b = eng(), eng()
    sa, sb = Shard(MODEL, 0, 1, N), Shard(MODEL, 2, N - 1, N)
    await a.ensure_shard(sa)
    await b.ensure_shard(sb)
    # perturb, then restore from the checkpoint
    for lw in a.runner.weights.layers.values():
      lw.ln1.mul_(0.5)
    await a.load_checkpoint(sa, str(tmp_path))
    await b.load_checkpoint(sb, str(tmp_path))
    h, st = await a.infer_tensor("q", sa, ids)
    out, _ = await b.infer_tensor("q", sb, h, st)
    assert np.allclose(np.asarray(ref, np.float32), np.asarray(out, np.float32), atol=1e-5)

  run(main())


def test_checkpoint_selection_rejects_mixed_partitions(tmp_path):
  """Files of one iteration from two runs with different layer splits overlap: loading must refuse
  instead of letting sort order decide which copy of the shared layers wins; one complete
  partition loads, a gap in the requested layers is reported."""
  from xotorch_support_jetson_amd.train.checkpoint import select_checkpoint_files
  d = tmp_path / MODEL
  d.mkdir()

  def touch(*names):
    for n in names:
      (d / n).write_bytes(b"")

  touch(f"000-001-of-{N:03d}-000004.safetensors", f"002-{N - 1:03d}-of-{N:03d}-000004.safetensors",
        f"000-{N - 1:03d}-of-{N:03d}-000002.safetensors")
  it, files = select_checkpoint_files(tmp_path, Shard(MODEL, 1, 2, N))
  assert it == 4 and [f.name[:7] for f in files] == ["000-001", f"002-{N - 1:03d}"]
  touch(f"000-002-of-{N:03d}-000004.safetensors")  # a 3-layer first stage from another run
  it, files = select_checkpoint_files(tmp_path, Shard(MODEL, 0, N - 1, N))  # iteration 4 overlaps: skipped
  assert it == 2 and [f.name[:7] for f in files] == [f"000-{N - 1:03d}"]
  (d / f"000-{N - 1:03d}-of-{N:03d}-000002.safetensors").rename(d / f"000-{N - 1:03d}-of-{N:03d}-000002.bak")
  with pytest.raises(ValueError, match="overlap"):  # no complete iteration left: the newest one's error
    select_checkpoint_files(tmp_path, Shard(MODEL, 0, N - 1, N))
  (d / f"000-{N - 1:03d}-of-{N:03d}-000002.bak").rename(d / f"000-{N - 1:03d}-of-{N:03d}-000002.safetensors")
  (d / f"000-002-of-{N:03d}-000004.safetensors").unlink()
  (d / f"002-{N - 1:03d}-of-{N:03d}-000004.safetensors").unlink()
  # iteration 4 now lacks layers 2..N-1 (one peer's save failed): the complete iteration 2 loads
  it, _ = select_checkpoint_files(tmp_path, Shard(MODEL, 0, N - 1, N))
  assert it == 2
  # ... and so does a first stage, although iteration 4 covers it: every stage of a ring that reloads from
  # one directory must resume from the SAME iteration; an explicit iteration is honoured
  assert select_checkpoint_files(tmp_path, Shard(MODEL, 0, 1, N))[0] == 2
  assert select_checkpoint_files(tmp_path, Shard(MODEL, 0, 1, N), iteration=4)[0] == 4
  with pytest.raises(FileNotFoundError, match="no file for layers"):
    select_checkpoint_files(tmp_path, Shard(MODEL, 1, 3, N), iteration=4)
  (d / f"000-{N - 1:03d}-of-{N:03d}-000002.safetensors").unlink()
  # no iteration covers the whole model (each host saved its own layers): the newest covering the shard
  assert select_checkpoint_files(tmp_path, Shard(MODEL, 0, 1, N))[0] == 4
  with pytest.raises(FileNotFoundError, match="no file for layers"):
    select_checkpoint_files(tmp_path, Shard(MODEL, 0, N - 1, N))


def test_concurrent_requests_are_batched():
  """Concurrent requests on one peer run as one batched forward (mixed prefill lengths, then
  decode) and give the same logits as one-at-a-time execution."""
  async def main():
    s = Shard(MODEL, 0, N - 1, N)
    rng = np.random.default_rng(5)
    prompts = [rng.integers(0, 500, size=(1, L)) for L in (5, 9, 3, 12)]
    solo = eng()
    ref = []
    for i, p in enumerate(prompts):
      out, _ = await solo.infer_tensor(f"s{i}", s, p)
      tok = np.array([[int(np.argmax(np.asarray(out)))]])
      out2, _ = await solo.infer_tensor(f"s{i}", s, tok)
      ref.append((np.asarray(out), np.asarray(out2)))
    b = eng()
    await b.ensure_shard(s)
    calls = []
    orig = b.runner.forward
    b.runner.forward = lambda rids, qlens, x: (calls.append(len(rids)), orig(rids, qlens, x))[1]
    outs = await asyncio.gather(*(b.infer_tensor(f"b{i}", s, p) for i, p in enumerate(prompts)))
    toks = [np.array([[int(np.argmax(np.asarray(o)))]]) for o, _ in outs]
    outs2 = await asyncio.gather(*(b.infer_tensor(f"b{i}", s, t) for i, t in enumerate(toks)))
    assert max(calls) > 1 and len(calls) < 2 * len(prompts)  # batched, not one forward per request
    for (r1, r2), (o1, _), (o2, _) in zip(ref, outs, outs2):
      # bf16 activations: a different batch composition changes fp32 GEMM blocking -> rounding-level diffs
      assert np.allclose(r1, np.asarray(o1), atol=5e-3) and np.allclose(r2, np.asarray(o2), atol=5e-3)

  run(main())


def test_moe_training_matches_inference_and_pipeline():
  """Mixtral-style MoE fine-tuning: the trainer's forward reproduces the inference path's logits, a
  two-stage pipeline step equals the single-stage step (router and expert weights included), loss falls,
  and the trained weights are written back into the inference shard (re-interleaved expert gate/up)."""
  moe, n = "tiny-mixtral", 4

  async def main():
    rng = np.random.default_rng(5)
    x = rng.integers(0, 64, size=(2, 10))
    y = np.roll(x, -1, 1)
    ln = np.array([10, 7])
    full = eng()
    fs = Shard(moe, 0, n - 1, n)
    out_inf, _ = await full.infer_tensor("q", fs, x[:1])
    tr = full._get_trainer()
    with torch.no_grad():
      logits = tr.forward(torch.as_tensor(x[:1])).float()[0, -1]
    ref = torch.as_tensor(np.asarray(out_inf)).float().reshape(-1)
    # whole model: bf16 differences in the attention path can flip a near-tied top-2 routing, so the
    # logits are compared by correlation; the MoE layer itself is compared exactly on one input
    assert torch.corrcoef(torch.stack([logits, ref]))[0, 1] > 0.99
    torch.manual_seed(0)
    xn = torch.randn(16, tr.c.hidden_size).bfloat16()
    h = torch.zeros(16, tr.c.hidden_size, dtype=torch.bfloat16)
    full.runner.model._moe(xn, full.runner.weights.layers[1], h)
    with torch.no_grad():
      mine = tr._moe(xn, 1).float()
    assert torch.allclose(mine, h.float(), atol=1e-3, rtol=2e-2), (mine - h.float()).abs().max()

    l_full, _ = await full.train("t", fs, x, y, ln)
    s0, s1 = eng(), eng()
    a, b = Shard(moe, 0, 1, n), Shard(moe, 2, n - 1, n)
    h = await s0.train_forward("t", a, x)
    l_split, g = await s1.train("t", b, h, y, ln)
    await s0.train("t", a, x, g, ln, loss="back_gradient")
    assert abs(l_full - l_split) < 1e-3
    tf, t0, t1 = full.trainer, s0.trainer, s1.trainer
    for k in ("0.router", "1.egu", "0.edown", "embed"):
      assert torch.allclose(tf.master[k], t0.master[k], atol=2e-6), k
    for k in ("2.router", "3.egu", "3.edown", "norm"):
      assert torch.allclose(tf.master[k], t1.master[k], atol=2e-6), k
    assert (tf.master["0.router"] != tf.master["0.router"].new_tensor(0)).any()

    full.lr = 3e-3
    tf.lr = 3e-3
    losses = [(await full.train("t", fs, x, y, ln))[0] for _ in range(10)]
    assert losses[-1] < losses[0] * 0.9, losses
    out2, _ = await full.infer_tensor("q2", fs, x[:1])  # syncs the trained weights into the shard
    with torch.no_grad():
      logits2 = tf.forward(torch.as_tensor(x[:1])).float()[0, -1]
    ref2 = torch.as_tensor(np.asarray(out2)).float().reshape(-1)
    assert torch.corrcoef(torch.stack([logits2, ref2]))[0, 1] > 0.99
    assert not torch.allclose(ref, ref2, atol=1e-3)

  run(main())


def test_step_token_budget_and_chunked_prefill(monkeypatch):
  """A step takes at most MAX_STEP_TOKENS new tokens; a longer prompt prefills alone in chunks with the
  same logits as one pass (chunked prefill reads the cached prefix)."""
  import xotorch_support_jetson_amd.inference.sharded_engine as SE

  async def main():
    s = Shard(MODEL, 0, N - 1, N)
    rng = np.random.default_rng(7)
    long_p = rng.integers(0, 500, size=(1, 45))
    ref_e = eng()
    ref, _ = await ref_e.infer_tensor("r", s, long_p)
    monkeypatch.setattr(SE, "MAX_STEP_TOKENS", 16)
    e = eng()
    await e.ensure_shard(s)
    calls = []
    orig = e.runner.forward
    e.runner.forward = lambda rids, qlens, x: (calls.append(sum(qlens)), orig(rids, qlens, x))[1]
    out, _ = await e.infer_tensor("r", s, long_p)
    assert calls == [16, 16, 13]
    assert np.allclose(np.asarray(ref), np.asarray(out), atol=5e-3)
    calls.clear()
    prompts = [rng.integers(0, 500, size=(1, L)) for L in (10, 5, 9, 3)]
    await asyncio.gather(*(e.infer_tensor(f"b{i}", s, p) for i, p in enumerate(prompts)))
    assert max(calls) <= 16 and sum(calls) == 27
  run(main())


def test_presampled_tokens_match_greedy():
  """With the sampling parameters in the step's state, the last shard draws each token with the forward;
  sample() returns it (greedy here: the argmax) without another executor trip."""
  async def main():
    s = Shard(MODEL, 0, N - 1, N)
    e = eng()
    rng = np.random.default_rng(11)
    prompts = [rng.integers(0, 500, size=(1, L)) for L in (6, 4, 9)]
    st = {"temperature": 0.0, "top_k": 35}
    outs = await asyncio.gather(*(e.infer_tensor(f"p{i}", s, p, st) for i, p in enumerate(prompts)))
    toks = await asyncio.gather(*(e.sample(o, temp=0.0, top_k=35) for o, _ in outs))
    for (o, _), t in zip(outs, toks):
      assert int(t[0]) == int(np.argmax(np.asarray(o)))
    assert e.stats.get("presampled", 0) == 3
    # a different temperature than the state's falls back to a real draw
    out, _ = await e.infer_tensor("q", s, prompts[0], st)
    t = await e.sample(out, temp=0.0, top_k=1)
    assert int(t[0]) == int(np.argmax(np.asarray(out))) and e.stats["presampled"] == 3
  run(main())


@pytest.mark.parametrize("model", ["tiny-deepseek-v2", "tiny-deepseek-v3"])
def test_deepseek_training_matches_inference_and_pipeline(model):
  """DeepSeek fine-tuning (MLA in its expanded form + DeepSeekMoE with shared experts, group-limited /
  noaux_tc routing): the trainer's forward reproduces the serving path's (absorbed MLA) logits, a two-stage
  pipeline step equals the single-stage step, loss falls, and the trained latent projections (kv_b split
  back into W_UK / W_UV), shared experts and router reach the inference shard."""
  n = 3

  async def main():
    rng = np.random.default_rng(7)
    x = rng.integers(0, 64, size=(2, 10))
    y = np.roll(x, -1, 1)
    ln = np.array([10, 7])
    full = eng()
    fs = Shard(model, 0, n - 1, n)
    out_inf, _ = await full.infer_tensor("q", fs, x[:1])
    tr = full._get_trainer()
    with torch.no_grad():
      logits = tr.forward(torch.as_tensor(x[:1])).float()[0, -1]
    ref = torch.as_tensor(np.asarray(out_inf)).float().reshape(-1)
    assert torch.corrcoef(torch.stack([logits, ref]))[0, 1] > 0.99
    li = next(i for i in range(n) if tr.c.moe_layer(i))
    torch.manual_seed(0)
    xn = torch.randn(16, tr.c.hidden_size).bfloat16()
    h = torch.zeros(16, tr.c.hidden_size, dtype=torch.bfloat16)
    full.runner.model._moe(xn, full.runner.weights.layers[li], h)
    with torch.no_grad():
      mine = tr._moe(xn, li).float()
    assert torch.allclose(mine, h.float(), atol=2e-3, rtol=2e-2), (mine - h.float()).abs().max()

    l_full, _ = await full.train("t", fs, x, y, ln)
    s0, s1 = eng(), eng()
    a, b = Shard(model, 0, 0, n), Shard(model, 1, n - 1, n)
    hh = await s0.train_forward("t", a, x)
    l_split, g = await s1.train("t", b, hh, y, ln)
    await s0.train("t", a, x, g, ln, loss="back_gradient")
    assert abs(l_full - l_split) < 1e-3
    tf, t0, t1 = full.trainer, s0.trainer, s1.trainer
    for k in ("0.qkv", "0.kvb", "0.kv_ln", "0.gu", "embed"):
      assert torch.allclose(tf.master[k], t0.master[k], atol=2e-6), k
    for k in ("1.router", "1.egu", "1.sh_gu", "2.kvb", "2.o", "norm"):
      assert torch.allclose(tf.master[k], t1.master[k], atol=2e-6), k
    if tr.c.q_lora_rank:
      assert torch.allclose(tf.master["1.qb"], t1.master["1.qb"], atol=2e-6)

    full.lr = 3e-3
    tf.lr = 3e-3
    losses = [(await full.train("t", fs, x, y, ln))[0] for _ in range(10)]
    assert losses[-1] < losses[0] * 0.9, losses
    out2, _ = await full.infer_tensor("q2", fs, x[:1])  # syncs the trained weights into the shard
    with torch.no_grad():
      logits2 = tf.forward(torch.as_tensor(x[:1])).float()[0, -1]
    ref2 = torch.as_tensor(np.asarray(out2)).float().reshape(-1)
    assert torch.corrcoef(torch.stack([logits2, ref2]))[0, 1] > 0.99
    assert not torch.allclose(ref, ref2, atol=1e-3)

  run(main())

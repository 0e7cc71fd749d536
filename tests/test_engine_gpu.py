"""GPU engine/trainer checks: HF parity through the HIP path (stream GEMM on shuffled weights, paged
attention kernels, HIP-graph decode), pipeline training on the HIP kernels vs the CPU reference path,
and the driver smoke."""
import asyncio

import numpy as np
import pytest
import torch

from xotorch_support_jetson_amd.download.shard_download import NoopShardDownloader
from xotorch_support_jetson_amd.inference.shard import Shard
from xotorch_support_jetson_amd.inference.sharded_engine import ShardedInferenceEngine

pytestmark = pytest.mark.gpu
MODEL, N = "tiny-llama", 4


def test_hf_parity_gpu(gpu, tmp_path):
  transformers = pytest.importorskip("transformers")
  from tests.test_hf_parity import _hf_model
  from xotorch_support_jetson_amd.models.config import load_config
  from xotorch_support_jetson_amd.models.weights import load_hf_weights
  from xotorch_support_jetson_amd.runtime.runner import ShardRunner
  # bf16 kernels vs the fp32 HF model on peaked attention (q weights x 6).  Phi-3's LongRoPE attention
  # factor (sqrt(3) here) sharpens the softmax so much that ANY bf16 pipeline leaves the fp32 model at the
  # later decode steps (our CPU path with bf16 weights: cos 0.977, tools/diag/phi3_gpu.py); there the
  # reference is that CPU bf16 path (its fp32 parity with HF: tests/test_hf_parity.py)
  bad = []
  for kind in ("llama", "qwen2", "phi3", "deepseek_v2", "deepseek_v3"):
    hf, d = _hf_model(kind, tmp_path)
    c = load_config(d)
    L = 40
    ids = torch.randint(0, c.vocab_size, (1, L + 4))
    s = Shard(kind, 0, c.num_layers - 1, c.num_layers)
    if kind == "phi3":
      rc = ShardRunner(c, s, "cpu", weights=load_hf_weights(d, c, s, dtype=torch.bfloat16), max_batch=4, max_ctx=128)
      ref = [rc.forward(["q"], [L], ids[0, :L].to(torch.int32)).float().view(-1)]
      ref += [rc.forward(["q"], [1], ids[0, t:t + 1].to(torch.int32)).float().view(-1) for t in range(L, L + 4)]
      ref = torch.stack([torch.zeros_like(ref[0])] * (L - 1) + ref)
    else:
      with torch.no_grad():
        ref = hf(ids).logits[0].float()
    r = ShardRunner(c, s, gpu, weights=load_hf_weights(d, c, s, device=gpu), max_batch=4, max_ctx=128)
    got = [r.forward(["q"], [L], ids[0, :L].to(torch.int32).to(gpu)).float().view(-1).cpu()]
    for t in range(L, L + 4):
      got.append(r.forward(["q"], [1], ids[0, t:t + 1].to(torch.int32).to(gpu)).float().view(-1).cpu())
    for k, g in enumerate(got):
      rr = ref[L - 1 + k]
      cos = torch.nn.functional.cosine_similarity(g, rr, dim=0).item()
      err = (g - rr).abs().max().item() / rr.abs().max().item()
      cmin, emax = (0.998, 0.1) if kind == "phi3" else (0.999, 6e-2)
      if not (cos > cmin and err < emax):
        bad.append((kind, k, cos, err))
  assert not bad, bad


def test_training_gpu_matches_cpu(gpu):
  async def main():
    x = np.random.default_rng(1).integers(0, 500, size=(2, 32))
    y = np.roll(x, -1, 1)
    ln = np.array([32, 20])
    from xotorch_support_jetson_amd.models.weights import copy_weights_into, random_weights
    from xotorch_support_jetson_amd.models.config import PRESETS
    out = {}
    a, b = Shard(MODEL, 0, 1, N), Shard(MODEL, 2, N - 1, N)
    for dev in ("cpu", "cuda:0"):
      e = ShardedInferenceEngine(NoopShardDownloader(), device=torch.device(dev))
      e2 = ShardedInferenceEngine(NoopShardDownloader(), device=torch.device(dev))
      await e.ensure_shard(a)
      await e2.ensure_shard(b)
      # random init is generated on the device (different streams on CPU and GPU): start both from the
      # CPU weights, written into the GPU engine's pre-shuffled layout in place
      for eng, sh in ((e, a), (e2, b)):
        copy_weights_into(eng.runner.weights, random_weights(PRESETS[MODEL], sh, "cpu", seed=0))
        eng.lr = 1e-3
      losses = []
      for _ in range(3):
        h = await e.train_forward("t", a, x)
        l, g = await e2.train("t", b, h, y, ln)
        await e.train("t", a, x, g, ln, loss="back_gradient")
        losses.append(l)
      logits, _ = await e2.infer_tensor("q", b, (await e.infer_tensor("q", a, x[:1]))[0])
      out[dev] = (losses, np.asarray(torch.as_tensor(logits).float().cpu(), np.float32))
    lc, lg = out["cpu"][0], out["cuda:0"][0]
    assert np.allclose(lc, lg, rtol=2e-2), (lc, lg)
    assert lg[-1] < lg[0]
    a_, b_ = out["cpu"][1].ravel(), out["cuda:0"][1].ravel()
    cos = float(np.dot(a_, b_) / np.linalg.norm(a_) / np.linalg.norm(b_))
    assert cos > 0.995  # trained weights were written back into the shuffled inference layout

  asyncio.run(main())


def test_graft_smoke(gpu):
  import __graft_entry__ as g
  g.smoke()


def test_llava_parity_gpu(gpu, tmp_path):
  """LLaVA through the GPU path (vision tower GEMMs on the kernel library, spliced image rows, HIP-graph
  decode) vs HF LlavaForConditionalGeneration in fp32."""
  pytest.importorskip("transformers")
  from tests.test_hf_parity import _hf_llava
  from xotorch_support_jetson_amd.models.config import load_config
  from xotorch_support_jetson_amd.models.vision import num_image_tokens
  from xotorch_support_jetson_amd.models.weights import load_hf_weights
  from xotorch_support_jetson_amd.runtime.runner import ShardRunner
  hf, d = _hf_llava(tmp_path)
  c = load_config(d)
  n_img = num_image_tokens(c)
  g = torch.Generator().manual_seed(0)
  ids = torch.cat([torch.tensor([1, 5, 6]), torch.full((n_img,), c.image_token_id), torch.randint(3, 298, (9,), generator=g)])
  pixels = torch.randn(1, 3, 56, 56, generator=g)
  L = ids.numel()
  with torch.no_grad():
    ref = hf(input_ids=ids[None], pixel_values=pixels).logits[0].float()
  s = Shard("llava", 0, c.num_layers - 1, c.num_layers)
  r = ShardRunner(c, s, gpu, weights=load_hf_weights(d, c, s, device=gpu), max_batch=4, max_ctx=128)
  feats = r.image_features(pixels)
  got = [r.forward(["q"], [L - 3], ids[:L - 3].to(torch.int32), image_embeds=feats).float().view(-1).cpu()]
  for t in range(L - 3, L):
    got.append(r.forward(["q"], [1], ids[t:t + 1].to(torch.int32)).float().view(-1).cpu())
  for k, gk in enumerate(got):
    rr = ref[L - 4 + k]
    cos = torch.nn.functional.cosine_similarity(gk, rr, dim=0).item()
    err = (gk - rr).abs().max().item() / rr.abs().max().item()
    assert cos > 0.999 and err < 6e-2, (k, cos, err)


def test_engine_concurrent_serving_gpu():
  """Many concurrent requests of mixed prompt lengths on the GPU engine (token-budgeted steps, chunked long
  prefill, several decode-graph buckets): greedy continuations equal one-at-a-time runs."""
  from xotorch_support_jetson_amd.inference.sharded_engine import ShardedInferenceEngine

  async def main():
    s = Shard(MODEL, 0, N - 1, N)
    rng = np.random.default_rng(9)
    prompts = [rng.integers(0, 500, size=(1, int(L))) for L in rng.integers(3, 300, size=24)]

    async def gen(e, rid, p, steps=5):
      out, _ = await e.infer_tensor(rid, s, p)
      toks = []
      for _ in range(steps):
        t = int(np.argmax(np.asarray(out.float().cpu() if hasattr(out, "float") else out)))
        toks.append(t)
        out, _ = await e.infer_tensor(rid, s, np.array([[t]]))
      return toks

    solo = ShardedInferenceEngine(NoopShardDownloader(), device=torch.device("cuda:0"))
    ref = [await gen(solo, f"s{i}", p) for i, p in enumerate(prompts)]
    both = ShardedInferenceEngine(NoopShardDownloader(), device=torch.device("cuda:0"))
    got = await asyncio.gather(*(gen(both, f"c{i}", p) for i, p in enumerate(prompts)))
    same = sum(a == b for a, b in zip(ref, got))
    assert same >= len(prompts) - 2, (same, ref, got)  # bf16 batch-composition rounding may flip a near-tie
  asyncio.run(main())


@pytest.mark.parametrize("model", ["tiny-llama", "tiny-deepseek-v2"])
def test_prefix_cache_gpu(gpu, model):
  """Prompt-prefix reuse on the HIP path (forked pages read by the prefill kernels, graph decode after):
  the reusing prompt's logits and its next decode step match a fresh engine's (MHA and MLA caches)."""
  from tests.test_prefix_cache import greedy, host, prompts

  async def main():
    a, b = prompts(2)
    n = 4 if model == "tiny-llama" else 3
    s = Shard(model, 0, n - 1, n)
    e = ShardedInferenceEngine(NoopShardDownloader(), device=gpu)
    out, st = await e.infer_tensor("A", s, a)
    for _ in range(2):
      out, st = await e.infer_tensor("A", s, greedy(out), st)
    outb, _ = await e.infer_tensor("B", s, b)
    assert e.prefix_cache.stats["hit_tokens"] == 128
    fresh = ShardedInferenceEngine(NoopShardDownloader(), device=gpu)
    await fresh.ensure_shard(s)
    fresh.prefix_cache = None
    ref, _ = await fresh.infer_tensor("B", s, b)
    x, y = torch.as_tensor(host(outb)).view(-1), torch.as_tensor(host(ref)).view(-1)
    assert torch.corrcoef(torch.stack([x, y]))[0, 1] > 0.999
    o2, _ = await e.infer_tensor("B", s, greedy(outb))
    r2, _ = await fresh.infer_tensor("B", s, greedy(ref))
    x, y = torch.as_tensor(host(o2)).view(-1), torch.as_tensor(host(r2)).view(-1)
    assert torch.corrcoef(torch.stack([x, y]))[0, 1] > 0.999

  asyncio.run(main())


def test_engine_loop_chained_gpu(gpu):
  """Engine-driven decode loop on the GPU -- device-chained steps (sampled ids handed to the next step in
  device memory, graph replay), requests joining a running chain and ending at different steps: greedy
  tokens equal the step-by-step path of a fresh engine."""
  from xotorch_support_jetson_amd.inference import sharded_engine as se

  async def main():
    s = Shard(MODEL, 0, N - 1, N)
    rng = np.random.default_rng(5)
    lens, want = (5, 40, 130, 9, 64, 300), (6, 11, 3, 17, 8, 12)
    prompts = [rng.integers(0, 500, size=(1, L)) for L in lens]

    ref_e = ShardedInferenceEngine(NoopShardDownloader(), device=gpu)
    ref = []
    for i, p in enumerate(prompts):
      out, _ = await ref_e.infer_tensor(f"r{i}", s, p)
      t = int(torch.as_tensor(out).float().argmax())
      toks = []
      for _ in range(want[i]):
        out, _ = await ref_e.infer_tensor(f"r{i}", s, np.array([[t]]))
        t = int(torch.as_tensor(out).float().argmax())
        toks.append(t)
      ref.append(toks)

    e = ShardedInferenceEngine(NoopShardDownloader(), device=gpu)
    got = {i: [] for i in range(len(prompts))}
    done = asyncio.Event()

    def emit(rid, tok):
      i = int(rid[1:])
      got[i].append(tok)
      if all(len(got[j]) >= want[j] for j in got):
        done.set()
      return len(got[i]) >= want[i]

    def stop(rid, tok):
      i = int(rid[1:])
      return len(got[i]) + 1 >= want[i]

    async def start(i):
      state = {"temperature": 0.0, "top_k": 35}
      logits, _ = await e.infer_tensor(f"c{i}", s, prompts[i], state)
      t = int(np.asarray(await e.sample(logits, 0.0, 35)).reshape(-1)[0])
      assert e.continue_locally(f"c{i}", s, t, dict(state), emit, stop=stop)

    await start(0)
    await start(1)
    await asyncio.sleep(0.05)  # the others join while a chain is running
    await asyncio.gather(*(start(i) for i in range(2, len(prompts))))
    await asyncio.wait_for(done.wait(), 120)
    assert e.stats.get("chained", 0) > 0
    same = sum(got[i] == ref[i] for i in range(len(prompts)))
    assert same >= len(prompts) - 1, (same, ref, got)  # bf16 batch-composition rounding may flip a near-tie
    for _ in range(100):
      if not e._draining:
        break
      await asyncio.sleep(0.01)
    assert not e._loops and not e._queue
    assert se.CHAIN

  asyncio.run(main())

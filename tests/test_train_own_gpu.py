"""`xot train` (the reference's protocol: Node -> engine.train -> ShardTrainer.step, reference
xotorch/orchestration/node.py:299-345, main.py:301-318) runs on the kernel library only: with the reference's
batch-size-1 ragged JSONL lengths (T not a multiple of 128) no vendor GEMM may run -- a dispatch mode that raises
on every aten GEMM op wraps the GPU engine's executor (and autograd's device threads, which inherit it) -- and
the losses and gradients still match the CPU path on the same weights."""
import asyncio

import numpy as np
import pytest
import torch
from torch.utils._python_dispatch import TorchDispatchMode

from xotorch_support_jetson_amd.download.shard_download import NoopShardDownloader
from xotorch_support_jetson_amd.inference.shard import Shard
from xotorch_support_jetson_amd.inference.sharded_engine import ShardedInferenceEngine

pytestmark = pytest.mark.gpu

GEMM_OPS = {"mm", "addmm", "bmm", "baddbmm", "addbmm", "matmul", "linear", "addmv", "mv", "dot", "_scaled_mm",
            "_addmm_activation", "tensordot", "einsum"}


class NoVendorGemm(TorchDispatchMode):
  """Raises on any aten GEMM / GEMV (hipBLASLt / rocBLAS) issued while active; counts the other ops."""

  def __init__(self):
    super().__init__()
    self.seen = []

  def __torch_dispatch__(self, func, types, args=(), kwargs=None):
    name = func.overloadpacket.__name__
    if name in GEMM_OPS and any(isinstance(a, torch.Tensor) and a.is_cuda for a in args):
      raise AssertionError(f"vendor GEMM on the train path: aten.{name}")
    self.seen.append(name)
    return func(*args, **(kwargs or {}))


def _guard(engine, mode):
  """Run every engine call inside `mode` on the engine's executor thread."""
  run = engine._run

  async def guarded(fn, *args):
    def call():
      with mode:
        return fn(*args)
    return await run(call)
  engine._run = guarded


@pytest.mark.parametrize("model", ["tiny-llama", "tiny-mixtral"])
def test_xot_train_ragged_no_vendor_gemm(gpu, model, monkeypatch):
  from xotorch_support_jetson_amd.models.config import PRESETS
  from xotorch_support_jetson_amd.models.weights import copy_weights_into, random_weights
  c = PRESETS[model]
  n = c.num_layers
  rng = np.random.default_rng(3)
  # batch size 1 with a ragged length (37 tokens), then 2 sequences padded to 53 with lengths 53 / 29
  batches = [rng.integers(0, c.vocab_size, size=(1, 37)), rng.integers(0, c.vocab_size, size=(2, 53))]
  lens = [np.array([37]), np.array([53, 29])]
  a, b = Shard(model, 0, n // 2 - 1, n), Shard(model, n // 2, n - 1, n)

  for fn in ("matmul", "mm", "addmm", "bmm"):  # the Python entry points too (belt and braces)
    real = getattr(torch, fn)

    def trap(*args, _real=real, _fn=fn, **kw):
      if any(isinstance(t, torch.Tensor) and t.is_cuda for t in args):
        raise AssertionError(f"torch.{_fn} on the train path")
      return _real(*args, **kw)
    monkeypatch.setattr(torch, fn, trap)

  async def run(dev):
    e, e2 = (ShardedInferenceEngine(NoopShardDownloader(), device=torch.device(dev)) for _ in range(2))
    await e.ensure_shard(a)
    await e2.ensure_shard(b)
    for eng, sh in ((e, a), (e2, b)):
      copy_weights_into(eng.runner.weights, random_weights(c, sh, "cpu", seed=0))
      eng.lr = 1e-3
    init = {k: v.float().cpu().clone() for k, v in e2._get_trainer().master.items()}
    mode = NoVendorGemm()
    if dev != "cpu":
      _guard(e, mode)
      _guard(e2, mode)
    losses, grads, m1 = [], [], None
    for x, ln in zip(batches * 2, lens * 2):
      y = np.roll(x, -1, 1)
      h = await e.train_forward("t", a, x)
      loss, g = await e2.train("t", b, h, y, ln)
      await e.train("t", a, x, g, ln, loss="back_gradient")
      losses.append(loss)
      grads.append(torch.as_tensor(g).float().reshape(-1))
      if m1 is None:  # AdamW's first moment after step 1: (1 - beta1) x the clipped gradient of every weight
        m1 = {k: v.float().cpu().clone() for k, v in e2._get_trainer().m.items()}
    tr = e2._get_trainer()
    if dev != "cpu":
      assert tr.fused_head() and "linear" not in mode.seen and len(mode.seen) > 100
    delta = {k: tr.master[k].float().cpu() - init[k] for k in tr.master}
    return losses, grads, delta, m1

  lc, gc, wc, mc = asyncio.run(run("cpu"))
  lg, gg, wg, mg = asyncio.run(run("cuda:0"))
  assert np.allclose(lc, lg, rtol=2e-2), (lc, lg)
  for x, y in zip(gc, gg):  # gradient wrt the stage input (the SendExample reply)
    cos = torch.nn.functional.cosine_similarity(x, y, dim=0).item()
    assert cos > 0.99, cos
  for k in mc:  # every weight gradient of the last stage (own-kernel dW, fused CE dHead, norm dw) vs CPU fp32
    d = ((mc[k] - mg[k]).abs().mean() / (mc[k].abs().mean() + 1e-12)).item()
    assert d < 0.05, (k, d)
  for k in wc:  # four AdamW steps from the same start: the updates (~ lr sign(m / sqrt(v)) early on, so elements
    # with near-zero gradients may flip) agree in the mean
    d = ((wc[k] - wg[k]).abs().mean() / (wc[k].abs().mean() + 1e-12)).item()
    assert d < 0.25, (k, d)


@pytest.mark.parametrize("N,K,gdt", [(256, 384, torch.bfloat16), (128, 1024, torch.float32)])
def test_adamw_tiled_matches_adamw_and_relayout(N, K, gdt):
  """The fused AdamW (csrc/train_ops.hip adamw_tiled) updates p / m / v as the plain kernel does and writes
  exactly shuffle(W) and shuffle(W^T) of its own bf16 result (the TrainWeight operand images)."""
  from xotorch_support_jetson_amd.ops._ext import require
  from xotorch_support_jetson_amd.ops.weights_layout import shuffle_for_stream
  C = require()
  dev = torch.device("cuda:0")
  torch.manual_seed(0)
  p0 = torch.randn(N, K, device=dev)
  g = (torch.randn(N, K, device=dev) * 0.1).to(gdt)
  m0, v0 = torch.randn(N, K, device=dev) * 0.01, torch.rand(N, K, device=dev) * 1e-3
  args = (1e-3, 0.9, 0.95, 1e-8, 0.1, 3, 0.7)
  p1, m1, v1, pb1 = p0.clone(), m0.clone(), v0.clone(), torch.empty(N, K, device=dev, dtype=torch.bfloat16)
  C.adamw(p1, g, m1, v1, pb1, *args)
  p2, m2, v2, pb2 = p0.clone(), m0.clone(), v0.clone(), torch.empty(N, K, device=dev, dtype=torch.bfloat16)
  ws = torch.empty(N, K, device=dev, dtype=torch.bfloat16)
  wts = torch.empty(K, N, device=dev, dtype=torch.bfloat16)
  C.adamw_tiled(p2, g, m2, v2, pb2, ws, wts, *args)
  torch.cuda.synchronize()
  for a, b in ((p1, p2), (m1, m2), (v1, v2)):
    assert torch.allclose(a, b, rtol=1e-6, atol=1e-7)
  assert (pb1.float() - pb2.float()).abs().max().item() <= 2 * (pb1.float().abs().max().item() * 2 ** -8)
  assert torch.equal(ws, shuffle_for_stream(pb2))
  assert torch.equal(wts, shuffle_for_stream(pb2.t().contiguous()))
  # without the plain copy the images are the same
  p3, m3, v3 = p0.clone(), m0.clone(), v0.clone()
  ws3, wts3 = torch.empty_like(ws), torch.empty_like(wts)
  C.adamw_tiled(p3, g, m3, v3, None, ws3, wts3, *args)
  assert torch.equal(ws3, ws) and torch.equal(wts3, wts)


@pytest.mark.parametrize("T", [300, 1024])
def test_silu_down_backward_matches_fp32(T):
  """A.SiluDownFn: y = (silu(gate) * up) . W_down^T + h and its backward (dA on the own tiles, silu_mul_bwd, the
  fused-accumulated dW_down) against fp32 torch autograd: dGU, dh and dW."""
  from xotorch_support_jetson_amd.train import autograd_ops as A
  dev = torch.device("cuda", 0)
  D, F = 384, 512
  torch.manual_seed(T)
  gu = (torch.randn(T, 2 * F, device=dev)).to(torch.bfloat16)
  w = (torch.randn(D, F, device=dev) / F ** 0.5).to(torch.bfloat16)
  h = torch.randn(T, D, device=dev).to(torch.bfloat16)
  dy = torch.randn(T, D, device=dev).to(torch.bfloat16)
  tw = A.TrainWeight(w)
  assert tw.ok
  acc = A.GradAcc("down", w)
  g, hh = gu.clone().requires_grad_(), h.clone().requires_grad_()
  y = A.silu_down_own(g, w, tw, acc, hh)
  y.backward(dy)
  A.join_dw_stream()
  torch.cuda.synchronize()
  gf, hf = gu.float().requires_grad_(), h.float().requires_grad_()
  wf = w.float().requires_grad_()
  yr = (torch.nn.functional.silu(gf[:, :F]) * gf[:, F:]) @ wf.t() + hf
  yr.backward(dy.float())
  for name, a, r in zip(("y", "dgu", "dh", "dW"), (y, g.grad, hh.grad, acc.buf), (yr, gf.grad, hf.grad, wf.grad)):
    assert rel_err(a, r) < 2e-2, (name, rel_err(a, r))


def rel_err(a, b):
  return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def test_embed_acc_matches_autograd():
  """A.EmbedAccFn: the embedding gradient of two micro-batches (repeated ids included) index-added into an fp32
  GradAcc equals autograd's summed dense gradient."""
  from xotorch_support_jetson_amd.train import autograd_ops as A
  dev = torch.device("cuda", 0)
  torch.manual_seed(0)
  V, D = 1000, 256
  w = (torch.randn(V, D, device=dev) * 0.1).to(torch.bfloat16)
  acc = A.GradAcc("embed", w)
  acc.buf = torch.empty(V, D, dtype=torch.float32, device=dev)
  wr = w.clone().requires_grad_()
  for mb in range(2):
    ids = torch.randint(0, 50, (3, 40), device=dev)  # many repeats
    dh = torch.randn(3, 40, D, device=dev).to(torch.bfloat16)
    A.embed_acc(ids, w.requires_grad_(), acc).backward(dh)
    torch.nn.functional.embedding(ids, wr).backward(dh)
  torch.cuda.synchronize()
  assert rel_err(acc.buf, wr.grad) < 1e-2
  assert acc.buf[50:].abs().max().item() == 0

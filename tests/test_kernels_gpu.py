"""Numerics of every HIP kernel against a plain PyTorch fp32 reference of the same op."""
import math

import pytest
import torch

from xotorch_support_jetson_amd.ops import kernels as K
from xotorch_support_jetson_amd.ops import reference as R
from xotorch_support_jetson_amd.ops.rope import build_cos_sin

pytestmark = pytest.mark.gpu


def rel_err(a, b):
  a, b = a.float(), b.float()
  return ((a - b).norm() / (b.norm() + 1e-12)).item()


@pytest.mark.parametrize("D", [896, 2048, 8192])
@pytest.mark.parametrize("with_res", [False, True])
def test_rmsnorm(gpu, D, with_res):
  torch.manual_seed(0)
  x = torch.randn(37, D, device=gpu, dtype=torch.bfloat16)
  w = torch.randn(D, device=gpu, dtype=torch.bfloat16)
  res = torch.randn_like(x) if with_res else None
  y, r = K.rmsnorm(x, w, 1e-5, res)
  yr, rr = R.rmsnorm(x, w, 1e-5, res)
  assert rel_err(y, yr) < 1e-2
  if with_res:
    assert torch.equal(r, rr)


def test_rmsnorm_bwd(gpu):
  torch.manual_seed(0)
  x = torch.randn(40, 2048, device=gpu, dtype=torch.bfloat16)
  w = torch.randn(2048, device=gpu, dtype=torch.bfloat16)
  dy = torch.randn_like(x)
  xr = x.float().requires_grad_()
  wr = w.float().requires_grad_()
  yr = xr * torch.rsqrt(xr.pow(2).mean(-1, keepdim=True) + 1e-5) * wr
  yr.backward(dy.float())
  from xotorch_support_jetson_amd.ops._ext import require
  dx = torch.empty_like(x)
  dw = torch.zeros(2048, device=gpu, dtype=torch.float32)
  require().rmsnorm_bwd(x, w, dy, dx, dw, 1e-5)
  assert rel_err(dx, xr.grad) < 2e-2
  assert rel_err(dw, wr.grad) < 1e-2
  # the residual stream's gradient joined in the same kernel (training's ResNormFn)
  res = torch.randn_like(x)
  dx2 = torch.empty_like(x)
  dw2 = torch.zeros(2048, device=gpu, dtype=torch.float32)
  require().rmsnorm_bwd(x, w, dy, dx2, dw2, 1e-5, res)
  assert rel_err(dx2, xr.grad + res.float()) < 2e-2
  assert torch.allclose(dw2, dw, rtol=1e-5, atol=1e-4)  # atomics: summation order varies


def test_multi_sumsq(gpu):
  """Gradient-clipping sum of squares over many tensors (bf16 and fp32, odd sizes, an unaligned view start):
  the fp32 sum of the per-tensor squared norms."""
  torch.manual_seed(0)
  from xotorch_support_jetson_amd.ops._ext import require
  ts = [torch.randn(n, device=gpu, dtype=torch.bfloat16) for n in (1, 7, 4096, 300_001, 2_100_000)]
  ts += [torch.randn(n, device=gpu, dtype=torch.float32) for n in (5, 65_537)]
  ts.append(torch.randn(1001, device=gpu, dtype=torch.bfloat16)[3:])  # data pointer not 16-byte aligned
  ts += [torch.randn(33, device=gpu, dtype=torch.bfloat16) for _ in range(70)]  # more than one batch of 64
  got = float(require().multi_sumsq(ts)[0])
  want = float(sum(t.float().pow(2).sum() for t in ts))
  assert abs(got - want) <= 1e-4 * want


def test_embedding_and_silu(gpu):
  torch.manual_seed(0)
  table = torch.randn(1000, 256, device=gpu, dtype=torch.bfloat16)
  ids = torch.randint(0, 1000, (33,), device=gpu)
  assert torch.equal(K.embedding(ids, table), table[ids])
  gu = torch.randn(17, 2 * 512, device=gpu, dtype=torch.bfloat16)
  assert rel_err(K.silu_mul(gu), R.silu_mul(gu)) < 1e-2


@pytest.mark.parametrize("M,N,Kd", [(1, 1024, 2048), (7, 2048, 4096), (16, 512, 896), (33, 1024, 4096),
                                    (64, 4096, 8192), (100, 1024, 2048), (128, 2048, 1024)])
def test_gemm_skinny(gpu, M, N, Kd):
  torch.manual_seed(0)
  x = torch.randn(M, Kd, device=gpu, dtype=torch.bfloat16)
  w = torch.randn(N, Kd, device=gpu, dtype=torch.bfloat16) / math.sqrt(Kd)
  y = K.gemm(x, w, algo=1)
  assert rel_err(y, R.linear(x, w)) < 1e-2
  yf = K.gemm(x, w, algo=1, out_dtype=torch.float32)
  assert rel_err(yf, R.linear(x, w)) < 1e-3


@pytest.mark.parametrize("H,T", [(16, 1), (16, 37), (16, 256), (128, 200)])
def test_gemm_batched_mla(gpu, H, T):
  """The MLA absorbed projections on gemm_batched (per-head pre-shuffled weights) vs fp32 bmm, reading the
  query heads in place from a strided [T, H dn | H dr] row and writing o as [T, H dv]; plus the stream_t
  layout round trip (prepare_for_decode -> _rowmajor, assign_weight)."""
  from xotorch_support_jetson_amd.ops._ext import require
  from xotorch_support_jetson_amd.models.weights import _rowmajor, assign_weight
  from xotorch_support_jetson_amd.ops.weights_layout import shuffle_for_stream
  torch.manual_seed(0)
  dn, dr, dv, L = 128, 64, 128, 512
  q = torch.randn(T, H * (dn + dr), device=gpu, dtype=torch.bfloat16)
  wuk = torch.randn(H, dn, L, device=gpu, dtype=torch.bfloat16) / math.sqrt(dn)
  wuv = torch.randn(H, dv, L, device=gpu, dtype=torch.bfloat16) / math.sqrt(L)
  wuk_s = torch.stack([shuffle_for_stream(wuk[h].t().contiguous()) for h in range(H)])
  wuv_s = torch.stack([shuffle_for_stream(wuv[h]) for h in range(H)])
  C = require()
  q_lat = torch.empty(H, T, L, device=gpu, dtype=torch.bfloat16)
  C.gemm_batched(q[:, :H * dn], dn, dn, wuk_s, q_lat, T * L, L, T)
  ref = torch.bmm(q[:, :H * dn].view(T, H, dn).transpose(0, 1).float(), wuk.float())
  assert rel_err(q_lat, ref) < 1e-2
  o_lat = torch.randn(H, T, L, device=gpu, dtype=torch.bfloat16)
  o = torch.empty(T, H * dv, device=gpu, dtype=torch.bfloat16)
  C.gemm_batched(o_lat.view(H * T, L), T * L, L, wuv_s, o, dv, H * dv, T)
  ref_o = torch.bmm(o_lat.float(), wuv.float().transpose(1, 2)).transpose(0, 1).reshape(T, H * dv)
  assert rel_err(o, ref_o) < 1e-2
  of = torch.empty(T, H * dv, device=gpu, dtype=torch.float32)
  C.gemm_batched(o_lat.view(H * T, L), T * L, L, wuv_s, of, dv, H * dv, T)
  assert rel_err(of, ref_o) < 1e-3
  wuk_s.xot_layout = "stream_t"
  assert torch.equal(_rowmajor(wuk_s), wuk)
  assign_weight(wuk_s, wuk * 2)
  assert torch.equal(_rowmajor(wuk_s), wuk * 2)


def test_gemm_epilogues(gpu):
  torch.manual_seed(0)
  M, Kd, Fd = 24, 1024, 512
  x = torch.randn(M, Kd, device=gpu, dtype=torch.bfloat16)
  w = torch.randn(2 * Fd, Kd, device=gpu, dtype=torch.bfloat16) / 32
  b = torch.randn(2 * Fd, device=gpu, dtype=torch.bfloat16)
  r = torch.randn(M, 2 * Fd, device=gpu, dtype=torch.bfloat16)
  y = K.gemm(x, w, bias=b, residual=r, epi="resid")
  assert rel_err(y, R.linear(x, w, b) + r.float()) < 1e-2
  # silu epilogue over 16-row interleaved gate/up
  ys = K.gemm(x, w, epi="silu")
  full = R.linear(x, w).view(M, Fd // 16, 2, 16)
  ref = (torch.nn.functional.silu(full[:, :, 0]) * full[:, :, 1]).reshape(M, Fd)
  assert rel_err(ys, ref) < 1e-2


@pytest.mark.parametrize("M,N,Kd", [(256, 1024, 1024), (300, 520, 2048), (1024, 2048, 4096)])
def test_gemm_tiled(gpu, M, N, Kd):
  torch.manual_seed(0)
  x = torch.randn(M, Kd, device=gpu, dtype=torch.bfloat16)
  w = torch.randn(N, Kd, device=gpu, dtype=torch.bfloat16) / math.sqrt(Kd)
  r = torch.randn(M, N, device=gpu, dtype=torch.bfloat16)
  assert rel_err(K.gemm(x, w, algo=2), R.linear(x, w)) < 1e-2
  assert rel_err(K.gemm(x, w, residual=r, epi="resid", algo=2), R.linear(x, w) + r.float()) < 1e-2


def _make_cache(n_pages, Hkv, Dh, device):
  kc = torch.randn(n_pages, Hkv, 64, Dh, device=device, dtype=torch.bfloat16)
  vc = torch.randn(n_pages, Hkv, Dh, 64, device=device, dtype=torch.bfloat16)
  return kc, vc


@pytest.mark.parametrize("H,Hkv,Dh,T,contig", [(32, 8, 64, 19, False), (64, 8, 128, 19, False), (14, 2, 64, 19, False),
                                               (32, 8, 128, 19, False), (64, 8, 128, 300, False),
                                               (32, 8, 128, 1000, True), (14, 2, 64, 257, True)])
def test_rope_kv_write(gpu, H, Hkv, Dh, T, contig):
  """T >= 256 runs the 64-token tiled kernel (V transposed through LDS), random or prefill-like contiguous slots."""
  torch.manual_seed(0)
  cs = build_cos_sin(Dh, 4096, 500000.0, {"rope_type": "llama3", "factor": 32.0, "low_freq_factor": 1.0,
                                          "high_freq_factor": 4.0, "original_max_position_embeddings": 8192},
                     device=gpu)
  qkv = torch.randn(T, (H + 2 * Hkv) * Dh, device=gpu, dtype=torch.bfloat16)
  pos = torch.randint(0, 4000, (T,), device=gpu, dtype=torch.int32)
  pages = max(10, -(-T // 64) + 2)
  slots = (torch.arange(T, device=gpu) + 37 if contig else torch.randperm(pages * 64, device=gpu)[:T]).to(torch.int64)
  slots[3] = -1
  kc = torch.zeros(pages, Hkv, 64, Dh, device=gpu, dtype=torch.bfloat16)
  vc = torch.zeros(pages, Hkv, Dh, 64, device=gpu, dtype=torch.bfloat16)
  kr, vr = kc.clone(), vc.clone()
  q = K.rope_kv_write(qkv, pos, cs, slots, kc, vc, H, Hkv)
  x = qkv.view(T, H + 2 * Hkv, Dh)
  qr = R.rope(x[:, :H], pos, cs)
  R.write_kv(R.rope(x[:, H:H + Hkv], pos, cs), x[:, H + Hkv:], slots, kr, vr)
  assert rel_err(q, qr) < 1e-2
  assert rel_err(kc, kr) < 1e-2
  assert torch.equal(vc, vr)


@pytest.mark.parametrize("H,Hkv,Dh,bias", [(64, 8, 128, False), (14, 2, 64, True)])
def test_splitk_rope_kv_write(gpu, H, Hkv, Dh, bias):
  """QKV split-K slabs -> RoPE + paged KV write in one kernel == bf16 reduce, then rope_kv_write."""
  from xotorch_support_jetson_amd.ops._ext import require
  C = require()
  torch.manual_seed(0)
  T, S = 19, 3
  N = (H + 2 * Hkv) * Dh
  cs = build_cos_sin(Dh, 4096, 500000.0, None, device=gpu)
  ws = torch.randn(S, T, N, device=gpu)
  b = torch.randn(N, device=gpu).to(torch.bfloat16) if bias else None
  qkv = (ws[0] + ws[1] + ws[2] + (b.float() if bias else 0.0)).to(torch.bfloat16)
  pos = torch.randint(0, 4000, (T,), device=gpu, dtype=torch.int32)
  slots = torch.randperm(10 * 64, device=gpu)[:T].to(torch.int64)
  slots[3] = -1
  caches = [(torch.zeros(10, Hkv, 64, Dh, device=gpu, dtype=torch.bfloat16),
             torch.zeros(10, Hkv, Dh, 64, device=gpu, dtype=torch.bfloat16)) for _ in range(2)]
  q1 = K.rope_kv_write(qkv, pos, cs, slots, caches[0][0], caches[0][1], H, Hkv)
  q2 = torch.empty(T, H, Dh, device=gpu, dtype=torch.bfloat16)
  C.splitk_rope_kv_write(ws, S, b, pos, cs, slots, q2, caches[1][0], caches[1][1], H, Hkv)
  assert rel_err(q2, q1) < 1e-2
  assert rel_err(caches[1][0], caches[0][0]) < 1e-2
  assert rel_err(caches[1][1], caches[0][1]) < 1e-2


@pytest.mark.parametrize("H,Hkv,Dh", [(64, 8, 128), (32, 8, 64), (14, 2, 64), (32, 4, 128)])
@pytest.mark.parametrize("ctx", [[1, 64, 65, 700], [2100, 5, 1300, 64]])
def test_attn_decode(gpu, H, Hkv, Dh, ctx):
  torch.manual_seed(0)
  B = len(ctx)
  maxb = 40
  kc, vc = _make_cache(B * maxb + 3, Hkv, Dh, gpu)
  bt = torch.randperm(B * maxb + 3, device=gpu)[:B * maxb].view(B, maxb).to(torch.int32).contiguous()
  cl = torch.tensor(ctx, device=gpu, dtype=torch.int32)
  q = torch.randn(B, H, Dh, device=gpu, dtype=torch.bfloat16)
  scale = 1 / math.sqrt(Dh)
  ref = R.attn_decode(q, kc, vc, bt, cl, scale)
  for algo in (0, 1, 2, 3, 5, 6):  # workgroup kernel; wave kernel without / with page prefetch (2 / 3: double
    # register set, 5 / 6: one set refilled per half), + nt loads
    for ppp in (1, 3, 4, 8, None):  # None: per-call choice from the batch
      if algo == 0 and ppp in (1, 3):
        continue
      ws = K.DecodeWorkspace(B, H, Dh, maxb * 64, gpu, pages_per_part=ppp, algo=algo)
      out = K.attn_decode(q, kc, vc, bt, cl, scale, ws)
      assert rel_err(out, ref) < 2e-2, (algo, ppp)
      again = K.attn_decode(q, kc, vc, bt, cl, scale, ws)
      assert torch.equal(again, out), (algo, ppp)


@pytest.mark.parametrize("H,Hkv,Dh", [(32, 8, 128), (32, 8, 64), (14, 2, 64)])
@pytest.mark.parametrize("ctx", [[700, 65, 1, 1024], [1], [512, 3]])
def test_attn_decode_auto_short_table(gpu, H, Hkv, Dh, ctx):
  """The default choice at small batch over a short block table (the workgroup kernel below 64 (sequence, KV head)
  pairs) against the fp32 reference."""
  torch.manual_seed(1)
  B, maxb = len(ctx), 16
  kc, vc = _make_cache(B * maxb + 3, Hkv, Dh, gpu)
  bt = torch.randperm(B * maxb + 3, device=gpu)[:B * maxb].view(B, maxb).to(torch.int32).contiguous()
  cl = torch.tensor(ctx, device=gpu, dtype=torch.int32)
  q = torch.randn(B, H, Dh, device=gpu, dtype=torch.bfloat16)
  ws = K.DecodeWorkspace(B, H, Dh, maxb * 64, gpu, algo=-1)
  assert ws.partition(B, Hkv, maxb)[2] in (0, 2)
  out = K.attn_decode(q, kc, vc, bt, cl, 1 / math.sqrt(Dh), ws)
  assert rel_err(out, R.attn_decode(q, kc, vc, bt, cl, 1 / math.sqrt(Dh))) < 2e-2


@pytest.mark.parametrize("algo", [1, 2])
@pytest.mark.parametrize("H,Hkv,Dh", [(32, 8, 64), (64, 8, 128), (14, 2, 64), (8, 8, 128), (32, 8, 128)])
@pytest.mark.parametrize("lens", [([5, 130, 1, 77], [5, 200, 64, 77]), ([300, 1000, 64], [300, 1100, 1000])])
def test_attn_prefill(gpu, H, Hkv, Dh, lens, algo, monkeypatch):
  """Causal varlen prefill from the paged cache, fresh prompts and chunks on top of a cached prefix; the
  second case spans several 256-row tiles per sequence (heaviest-first order, waves past the causal edge)."""
  monkeypatch.setattr(K, "PREFILL_ALGO", algo)
  torch.manual_seed(0)
  qlens, ctxs = lens
  B = len(qlens)
  maxb = max(-(-c // 64) for c in ctxs) + 1
  kc, vc = _make_cache(B * maxb, Hkv, Dh, gpu)
  bt = torch.randperm(B * maxb, device=gpu).view(B, maxb).to(torch.int32).contiguous()
  cu = torch.tensor([0] + list(torch.tensor(qlens).cumsum(0)), device=gpu, dtype=torch.int32)
  cl = torch.tensor(ctxs, device=gpu, dtype=torch.int32)
  q = torch.randn(sum(qlens), H, Dh, device=gpu, dtype=torch.bfloat16)
  scale = 1 / math.sqrt(Dh)
  out = K.attn_prefill(q, kc, vc, bt, cu, cl, max(qlens), scale)
  ref = R.attn_prefill(q, kc, vc, bt, cu, cl, scale)
  assert rel_err(out, ref) < 2e-2


def test_sample_greedy_and_topk(gpu):
  torch.manual_seed(0)
  B, V = 6, 128256
  logits = torch.randn(B, V, device=gpu) * 3
  so = torch.tensor([1234, 0], device=gpu, dtype=torch.int64)
  greedy = K.sample(logits, torch.zeros(B, device=gpu), 35, so)
  assert torch.equal(greedy.cpu(), logits.argmax(-1).int().cpu())
  temps = torch.full((B,), 0.8, device=gpu)
  mask = R.topk_mask(logits, 35)
  seen = set()
  for step in range(20):
    so[1] = step
    tok = K.sample(logits, temps, 35, so)
    assert bool(mask[torch.arange(B, device=gpu), tok.long()].all())
    seen.add(tuple(tok.tolist()))
  assert len(seen) > 1  # actually random across offsets
  # top_k = 1 is greedy even with temperature
  assert torch.equal(K.sample(logits, temps, 1, so).cpu(), greedy.cpu())


def test_sample_split_path_matches_single_block(gpu):
  """Small batches take the two-stage (64 chunk workgroups + merge) path; for the same seed and row
  index it must pick the same tokens as the one-workgroup-per-row path used for large batches."""
  torch.manual_seed(1)
  V = 128256
  small = torch.randn(6, V, device=gpu) * 3
  big = torch.cat([small, torch.randn(60, V, device=gpu) * 3])  # 66 rows -> single-block path
  for temp, k in ((0.0, 35), (0.7, 35), (1.0, 64), (0.5, 7)):
    so = torch.tensor([99, 5], device=gpu, dtype=torch.int64)
    a = K.sample(small, torch.full((6,), temp, device=gpu), k, so)
    b = K.sample(big, torch.full((66,), temp, device=gpu), k, so)
    assert torch.equal(a.cpu(), b[:6].cpu()), (temp, k)


@pytest.mark.parametrize("algo", [1, 2])
def test_sample_algos_match_single_block(gpu, algo):
  """Chunk candidates + merge (1) and the two-pass candidate filter (2) must pick exactly the tokens of
  the 5-pass one-workgroup-per-row path (0), including rows whose ties overflow the candidate list."""
  from xotorch_support_jetson_amd.ops._ext import require
  C = require()
  torch.manual_seed(2)
  V = 128256
  lg = torch.randn(70, V, device=gpu) * 3
  lg[3] = 0.0  # every logit tied: filter overflows -> exact fallback
  lg[4] = torch.randint(0, 3, (V,), device=gpu).float()  # heavy ties at the cut
  for temp, k in ((0.0, 35), (0.7, 35), (1.0, 64), (0.5, 7), (0.9, 1)):
    temps = torch.full((70,), temp, device=gpu)
    so = torch.tensor([99, 5], device=gpu, dtype=torch.int64)
    a = torch.empty(70, dtype=torch.int32, device=gpu)
    b = torch.empty_like(a)
    C.sample(lg, temps, k, so, a, 0)
    C.sample(lg, temps, k, so, b, algo)
    rows = torch.arange(70) if algo == 2 or temp == 0.0 or k == 1 else torch.tensor([r for r in range(70) if r not in (3, 4)])
    # (the chunk path keeps at most k tied candidates per chunk, so it may differ on rows tied at the cut)
    assert torch.equal(a.cpu()[rows], b.cpu()[rows]), (temp, k)


def test_topk_cand(gpu):
  """Per-row top-k (value, index) candidates of a vocab slice (split LM head) == torch.topk's set."""
  torch.manual_seed(3)
  B, V, k, kc = 37, 64000, 35, 64
  lg = torch.randn(B, V, device=gpu) * 3
  lg[5] = 0.0  # all tied: the exact fallback path, any k of them
  vals, idx = K.topk_cand(lg, k, kc)
  ref_v, _ = torch.topk(lg, k, dim=-1)
  assert torch.equal(idx[:, k:].cpu(), torch.full((B, kc - k), -1, dtype=torch.int32))
  assert bool(torch.isinf(vals[:, k:]).all())
  got_v = torch.sort(vals[:, :k], dim=-1, descending=True).values
  assert torch.equal(got_v, ref_v)
  # values are the logits at the returned indices, indices distinct
  assert torch.equal(lg.gather(1, idx[:, :k].long()), vals[:, :k])
  assert all(len(set(r)) == k for r in idx[:, :k].tolist())


def test_sample_split_distribution(gpu):
  base = torch.full((128256,), -30.0, device=gpu)
  base[[10, 70000, 128000]] = torch.tensor([2.0, 1.0, 0.5], device=gpu)
  lg = base.expand(8, -1).contiguous()
  counts = torch.zeros(128256, device=gpu)
  for off in range(250):
    tok = K.sample(lg, torch.ones(8, device=gpu), 3, torch.tensor([3, off], device=gpu, dtype=torch.int64))
    counts += torch.bincount(tok.long(), minlength=128256).float()
  c = counts.cpu() / counts.sum().cpu()
  p = torch.softmax(torch.tensor([2.0, 1.0, 0.5]), 0)
  assert abs(float(c[10]) - float(p[0])) < 0.03 and abs(float(c[70000]) - float(p[1])) < 0.03
  assert float(c[10] + c[70000] + c[128000]) == 1.0


def test_sample_distribution(gpu):
  # exponential race == categorical(softmax(l / T)) restricted to top-k
  logits = torch.tensor([[2.0, 1.0, 0.5, 0.0, -1.0] + [-30.0] * 59], device=gpu)
  B = 4096
  lg = logits.expand(B, -1).contiguous()
  so = torch.tensor([7, 3], device=gpu, dtype=torch.int64)
  tok = K.sample(lg, torch.ones(B, device=gpu), 3, so)
  counts = torch.bincount(tok.long(), minlength=64).float().cpu() / B
  p = torch.softmax(torch.tensor([2.0, 1.0, 0.5]), 0)
  assert counts[3:].sum() == 0
  assert torch.allclose(counts[:3], p, atol=0.03)


@pytest.mark.parametrize("V", [50000, 50001, 512])
def test_cross_entropy_fp32_logits(gpu, V):
  """fp32 logits (the fused LM head's chunks): the 16-byte vector kernels (V % 8 == 0) and the scalar fallback."""
  from xotorch_support_jetson_amd.ops._ext import require
  C = require()
  torch.manual_seed(V)
  T = 7
  x = torch.randn(T, V, device=gpu) * 3
  tgt = torch.randint(0, V, (T,), device=gpu, dtype=torch.int32)
  tgt[1] = -100
  tgt[4] = V - 1
  loss, lse = torch.empty(T, device=gpu), torch.empty(T, device=gpu)
  C.ce_fwd(x, tgt, loss, lse)
  ref = torch.nn.functional.cross_entropy(x, tgt.long(), ignore_index=-100, reduction="none")
  assert torch.allclose(loss, ref, atol=1e-3, rtol=1e-4)
  dx = torch.empty(T, V, device=gpu, dtype=torch.bfloat16)
  C.ce_bwd(x, tgt, lse, torch.full((T,), 0.25, device=gpu), dx)
  xr = x.clone().requires_grad_()
  (torch.nn.functional.cross_entropy(xr, tgt.long(), ignore_index=-100, reduction="none") * 0.25).sum().backward()
  assert rel_err(dx, xr.grad) < 1e-2
  assert dx[1].abs().max().item() == 0


def test_cross_entropy_and_adamw(gpu):
  torch.manual_seed(0)
  from xotorch_support_jetson_amd.ops._ext import require
  C = require()
  T, V = 9, 50000
  x = torch.randn(T, V, device=gpu, dtype=torch.bfloat16)
  tgt = torch.randint(0, V, (T,), device=gpu, dtype=torch.int32)
  tgt[2] = -100
  loss, lse = torch.empty(T, device=gpu), torch.empty(T, device=gpu)
  C.ce_fwd(x, tgt, loss, lse)
  lr_, lser = R.cross_entropy(x, tgt)
  assert torch.allclose(loss, lr_, atol=1e-3, rtol=1e-4)
  dx = torch.empty_like(x)
  C.ce_bwd(x, tgt, lse, torch.full((T,), 0.5, device=gpu), dx)
  xr = x.float().requires_grad_()
  l = torch.nn.functional.cross_entropy(xr, tgt.long(), ignore_index=-100, reduction="none")
  (l * 0.5).sum().backward()
  assert rel_err(dx, xr.grad) < 1e-2
  # AdamW vs torch.optim.AdamW
  p = torch.randn(1000, device=gpu)
  g = torch.randn(1000, device=gpu)
  m, v = torch.zeros_like(p), torch.zeros_like(p)
  pt = p.clone().requires_grad_()
  opt = torch.optim.AdamW([pt], lr=1e-2, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1)
  for step in range(1, 4):
    C.adamw(p, g, m, v, None, 1e-2, 0.9, 0.95, 1e-8, 0.1, step, 1.0)
    pt.grad = g.clone()
    opt.step()
  assert torch.allclose(p, pt.detach(), atol=1e-5)


@pytest.mark.parametrize("M", [1, 5, 16, 33, 64, 100, 128, 200, 256, 300, 513])
@pytest.mark.parametrize("epi,ntw,splits", [("none", 1, 1), ("none", 2, 1), ("none", 1, 4), ("resid", 1, 2),
                                            ("silu", 2, 1), ("silu", 2, 2), ("none", 4, 1), ("silu", 4, 2),
                                            ("resid", 4, 2), ("resid", 2, 8), ("silu", 2, 8)])
def test_gemm_stream(gpu, M, epi, ntw, splits):
  from xotorch_support_jetson_amd.ops._ext import require
  torch.manual_seed(0)
  N, Kd = 1024, 2048
  x = torch.randn(M, Kd, device=gpu, dtype=torch.bfloat16)
  w = torch.randn(N, Kd, device=gpu, dtype=torch.bfloat16) / math.sqrt(Kd)
  b = torch.randn(N, device=gpu, dtype=torch.bfloat16)
  r = torch.randn(M, N, device=gpu, dtype=torch.bfloat16)
  ws = torch.empty(splits * M * N, device=gpu, dtype=torch.float32)
  full = R.linear(x, w, b)
  if epi == "silu":
    f = full.view(M, N // 32, 2, 16)
    ref = (torch.nn.functional.silu(f[:, :, 0]) * f[:, :, 1]).reshape(M, N // 2)
    y = torch.empty(M, N // 2, device=gpu, dtype=torch.bfloat16)
  elif epi == "resid":
    ref = full + r.float()
    y = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
  else:
    ref = full
    y = torch.empty(M, N, device=gpu, dtype=torch.float32)
  require().gemm_stream(x, w, y, b, r if epi == "resid" else None, ws, K.EPI[epi], ntw, splits, False)
  assert rel_err(y, ref) < 1e-2
  if True:  # pre-shuffled layout, every M (M > 128 runs the XCD-paired 128-row blocks)
    from xotorch_support_jetson_amd.ops.weights_layout import shuffle_for_stream
    y2 = torch.empty_like(y)
    require().gemm_stream(x, shuffle_for_stream(w), y2, b, r if epi == "resid" else None, ws, K.EPI[epi], ntw,
                          splits, True)
    assert rel_err(y2, ref) < 1e-2


@pytest.mark.parametrize("Kd,N,epi,ntw,splits,s_in,with_bias", [
    (2048, 1024, "none", 1, 4, 4, False), (2048, 1024, "none", 2, 2, 2, True), (4096, 2048, "silu", 2, 1, 4, False),
    (4096, 2048, "silu", 2, 4, 1, True), (8192, 1024, "none", 2, 4, 4, False), (4096, 768, "none", 1, 1, 3, False),
    (4096, 1024, "none", 2, 4, 8, True), (8192, 2048, "silu", 2, 1, 6, False)])
def test_gemm_stream_norm(gpu, Kd, N, epi, ntw, splits, s_in, with_bias):
  """Batch-1 GEMM with the RMSNorm of a pending split-K residual sum in its prologue (gemm_stream_norm) against the
  unfused pair (splitk_resid_rmsnorm, then gemm_stream on its output): the same arithmetic in the same order, so
  the summed residual row and the GEMM output are bitwise equal."""
  from xotorch_support_jetson_amd.ops._ext import require
  from xotorch_support_jetson_amd.ops.weights_layout import shuffle_for_stream
  C = require()
  torch.manual_seed(Kd + N + s_in)
  h = torch.randn(1, Kd, device=gpu, dtype=torch.bfloat16)
  ws_in = torch.randn(s_in * Kd, device=gpu, dtype=torch.float32) * 0.3
  bias_in = torch.randn(Kd, device=gpu, dtype=torch.bfloat16) if with_bias else None
  lnw = (1 + 0.1 * torch.randn(Kd, device=gpu)).to(torch.bfloat16)
  w = shuffle_for_stream(torch.randn(N, Kd, device=gpu, dtype=torch.bfloat16) / math.sqrt(Kd))
  b = torch.randn(N, device=gpu, dtype=torch.bfloat16) if with_bias else None
  ncol = N // 2 if epi == "silu" else N
  # unfused: slab reduce + residual + norm, then the stream GEMM on the normalised row
  h_ref = h.clone()
  xn = torch.empty_like(h)
  C.splitk_resid_rmsnorm(ws_in, s_in, bias_in, h_ref, lnw, xn, 1e-5)
  ws = torch.empty(max(splits, 1) * N, device=gpu, dtype=torch.float32)
  y_ref = torch.empty(1, ncol, device=gpu, dtype=torch.bfloat16)
  C.gemm_stream(xn, w, y_ref, b, None, ws, K.EPI[epi], ntw, splits, True)
  # fused
  hout = torch.full_like(h, 7.0)
  y = torch.empty_like(y_ref)
  C.gemm_stream_norm(w, y, b, torch.empty_like(ws), K.EPI[epi], ntw, splits, True, h, ws_in, s_in, bias_in, lnw, hout,
                     1e-5)
  assert torch.equal(hout, h_ref)
  assert torch.equal(y, y_ref), (y.float() - y_ref.float()).abs().max().item()
  # the residual buffer the prologue read is untouched
  h2 = h.clone()
  C.gemm_stream_norm(w, y, b, torch.empty_like(ws), K.EPI[epi], ntw, splits, True, h, ws_in, s_in, bias_in, lnw, hout,
                     1e-5)
  assert torch.equal(h, h2)


def test_fp8_layout_roundtrip(gpu):
  from xotorch_support_jetson_amd.ops.weights_layout import (dequant_stream8, quantize_fp8_rows, shuffle_for_stream8,
                                                             unshuffle_from_stream8)
  w = torch.randn(256, 512, device=gpu) / 20
  q, sc = quantize_fp8_rows(w)
  assert torch.equal(unshuffle_from_stream8(shuffle_for_stream8(q)), q)
  deq = dequant_stream8(shuffle_for_stream8(q), sc, torch.float32)
  assert rel_err(deq, w) < 0.04  # e4m3: 3 mantissa bits
  assert float((q.view(torch.float8_e4m3fn).float().abs().amax(1) - 448).abs().max()) == 0  # row absmax -> 448


@pytest.mark.parametrize("M", [1, 5, 16, 33, 100, 128, 200])
@pytest.mark.parametrize("epi,ntw,splits", [("none", 1, 1), ("none", 2, 4), ("resid", 1, 2), ("silu", 2, 1),
                                            ("silu", 4, 2), ("none", 4, 1), ("resid", 2, 8)])
def test_gemm_stream8(gpu, M, epi, ntw, splits):
  """Weight-only FP8 stream GEMM against the fp32 product with the dequantised weight (the kernel widens
  e4m3 to bf16 exactly, so only accumulation order and the bf16 output differ)."""
  from xotorch_support_jetson_amd.ops._ext import require
  from xotorch_support_jetson_amd.ops.weights_layout import dequant_stream8, quantize_fp8_rows, shuffle_for_stream8
  torch.manual_seed(0)
  N, Kd = 1024, 2048
  x = torch.randn(M, Kd, device=gpu, dtype=torch.bfloat16)
  w = torch.randn(N, Kd, device=gpu, dtype=torch.bfloat16) / math.sqrt(Kd)
  q, sc = quantize_fp8_rows(w)
  w8 = shuffle_for_stream8(q)
  b = torch.randn(N, device=gpu, dtype=torch.bfloat16)
  r = torch.randn(M, N, device=gpu, dtype=torch.bfloat16)
  ws = torch.empty(splits * M * N, device=gpu, dtype=torch.float32)
  full = x.float() @ dequant_stream8(w8, sc, torch.float32).t() + b.float()
  if epi == "silu":
    f = full.view(M, N // 32, 2, 16)
    ref = (torch.nn.functional.silu(f[:, :, 0]) * f[:, :, 1]).reshape(M, N // 2)
    y = torch.empty(M, N // 2, device=gpu, dtype=torch.bfloat16)
  elif epi == "resid":
    ref = full + r.float()
    y = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
  else:
    ref = full
    y = torch.empty(M, N, device=gpu, dtype=torch.float32)
  require().gemm_stream8(x, w8, sc, y, b, r if epi == "resid" else None, ws, K.EPI[epi], ntw, splits)
  assert rel_err(y, ref) < 1e-2


def test_linear_fp8_dispatch(gpu):
  """ops.linear on a "stream8" weight: FP8 stream GEMM for decode-shaped M, widened bf16 GEMM above."""
  from xotorch_support_jetson_amd.ops.linear import linear, to_rowmajor, to_stream8_layout
  torch.manual_seed(1)
  w = torch.randn(512, 1024, device=gpu, dtype=torch.bfloat16) / 32
  w8 = to_stream8_layout(w)
  assert w8.dtype == torch.uint8 and w8.xot_layout == "stream8"
  wd = to_rowmajor(w8)
  for M in (1, 64, 600):
    x = torch.randn(M, 1024, device=gpu, dtype=torch.bfloat16)
    assert rel_err(linear(x, w8), x.float() @ wd.float().t()) < 1e-2
    assert rel_err(linear(x, w8), x.float() @ w.float().t()) < 5e-2  # quantisation error


@pytest.mark.parametrize("M", [1, 33, 200])
@pytest.mark.parametrize("Kd", [128, 384, 1408])
@pytest.mark.parametrize("epi", ["none", "silu"])
def test_gemm_stream_odd_chunks(gpu, M, Kd, epi):
  """An odd number of 128-deep k-chunks (single-chunk tail; e.g. DeepSeek-V2-Lite's 1408-wide experts)."""
  from xotorch_support_jetson_amd.ops._ext import require
  from xotorch_support_jetson_amd.ops.weights_layout import shuffle_for_stream
  torch.manual_seed(Kd + M)
  N = 512
  x = torch.randn(M, Kd, device=gpu, dtype=torch.bfloat16)
  w = torch.randn(N, Kd, device=gpu, dtype=torch.bfloat16) / math.sqrt(Kd)
  full = R.linear(x, w, None)
  if epi == "silu":
    f = full.view(M, N // 32, 2, 16)
    ref = (torch.nn.functional.silu(f[:, :, 0]) * f[:, :, 1]).reshape(M, N // 2)
  else:
    ref = full
  for shuf in (False, True):
    y = torch.empty(M, N // 2 if epi == "silu" else N, device=gpu, dtype=torch.bfloat16)
    require().gemm_stream(x, shuffle_for_stream(w) if shuf else w, y, None, None, None, K.EPI[epi], 2, 1, shuf)
    assert rel_err(y, ref) < 1e-2, shuf


@pytest.mark.parametrize("M", [1, 77, 256, 300, 512, 700, 2100, 4100])
@pytest.mark.parametrize("epi,bn,splits", [("none", 256, 1), ("none", 128, 1), ("resid", 256, 1), ("silu", 256, 1),
                                           ("silu", 128, 1), ("none", 256, 3), ("resid", 128, 2), ("silu", 256, 5),
                                           ("none", 1256, 1), ("resid", 1256, 1), ("silu", 1256, 1), ("none", 1256, 3),
                                           ("resid", 1256, 4), ("none", 224, 1), ("silu", 224, 1), ("resid", 224, 2),
                                           ("silu", 224, 3), ("none", 2240256, 1), ("silu", 1920256, 1),
                                           ("resid", 1600128, 2), ("silu", 2240128, 1), ("none", 1920128, 3),
                                           ("none", 2256, 1), ("silu", 2256, 1), ("resid", 2256, 3), ("none", 2256, 5),
                                           ("none", 1922256, 1), ("silu", 1922256, 1), ("resid", 1922256, 3),
                                           ("none", 1922256, 5)])
def test_gemm_big(gpu, M, epi, bn, splits):
  """Large-M LDS-DMA GEMM on the pre-shuffled layout vs the fp32 reference: masked row tiles, both
  column tilings, uneven split-K ranges, every epilogue, fp32 and bf16 outputs."""
  from xotorch_support_jetson_amd.ops._ext import require
  from xotorch_support_jetson_amd.ops.weights_layout import shuffle_for_stream
  torch.manual_seed(M + bn + splits)
  N, Kd = 1024, 1280  # 20 k stages: splits of 3 and 5 get unequal ranges
  x = torch.randn(M, Kd, device=gpu, dtype=torch.bfloat16)
  w = torch.randn(N, Kd, device=gpu, dtype=torch.bfloat16) / math.sqrt(Kd)
  b = torch.randn(N, device=gpu, dtype=torch.bfloat16)
  r = torch.randn(M, N, device=gpu, dtype=torch.bfloat16)
  ws = torch.empty(splits * M * N, device=gpu, dtype=torch.float32)
  full = R.linear(x, w, b)
  if epi == "silu":
    f = full.view(M, N // 32, 2, 16)
    ref = (torch.nn.functional.silu(f[:, :, 0]) * f[:, :, 1]).reshape(M, N // 2)
    y = torch.empty(M, N // 2, device=gpu, dtype=torch.bfloat16)
  elif epi == "resid":
    ref = full + r.float()
    y = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
  else:
    ref = full
    y = torch.empty(M, N, device=gpu, dtype=torch.float32)
  require().gemm_big(x, shuffle_for_stream(w), y, b, r if epi == "resid" else None, ws, K.EPI[epi], bn, splits)
  assert rel_err(y, ref) < 1e-2


@pytest.mark.parametrize("N", [3648, 1088, 320])
@pytest.mark.parametrize("epi,bn,splits", [("none", 256, 1), ("none", 128, 1), ("none", 1256, 1), ("resid", 256, 1),
                                           ("silu", 128, 1), ("none", 256, 3), ("resid", 1256, 2), ("silu", 224, 1),
                                           ("none", 224, 1), ("resid", 1600256, 1), ("silu", 2240128, 2)])
def test_gemm_big_column_tail(gpu, N, epi, bn, splits):
  """N not a multiple of the column tile (DeepSeek-V2-Lite's fused A projection is 3648 wide): the last
  column tile re-reads the last weight row group and masks its stores -- columns past N stay untouched."""
  from xotorch_support_jetson_amd.ops._ext import require
  from xotorch_support_jetson_amd.ops.weights_layout import shuffle_for_stream
  torch.manual_seed(N + bn)
  M, Kd = 300, 1024
  x = torch.randn(M, Kd, device=gpu, dtype=torch.bfloat16)
  w = torch.randn(N, Kd, device=gpu, dtype=torch.bfloat16) / math.sqrt(Kd)
  r = torch.randn(M, N, device=gpu, dtype=torch.bfloat16)
  ws = torch.empty(splits * M * N, device=gpu, dtype=torch.float32)
  full = R.linear(x, w)
  Ny = N // 2 if epi == "silu" else N
  if epi == "silu":
    f = full.view(M, N // 32, 2, 16)
    ref = (torch.nn.functional.silu(f[:, :, 0]) * f[:, :, 1]).reshape(M, Ny)
  else:
    ref = full + r.float() if epi == "resid" else full
  buf = torch.full((M, Ny + 64), 7.0, device=gpu, dtype=torch.bfloat16)
  y = buf[:, :Ny]
  require().gemm_big(x, shuffle_for_stream(w), y, None, r if epi == "resid" else None, ws, K.EPI[epi], bn, splits)
  assert rel_err(y, ref) < 1e-2
  assert bool((buf[:, Ny:] == 7.0).all())


@pytest.mark.parametrize("M", [256, 300, 1024, 2100])
@pytest.mark.parametrize("epi,f32,splits", [("none", False, 1), ("none", True, 1), ("resid", False, 1),
                                            ("silu", False, 1), ("none", True, 3), ("silu", False, 2),
                                            ("resid", False, 4)])
def test_gemm_w4(gpu, M, epi, f32, splits):
  """Four-wave 256 x 256 tile (tile code 4256, csrc/gemm_w4.hip: swapped MFMA operands, permuted weight-row reads
  for 16-B stores, branch-free k loop) vs the fp32 reference: masked row tiles, every epilogue with a bias, fp32
  out, uneven split-K ranges (slabs reduced by the split-K reduce kernel)."""
  from xotorch_support_jetson_amd.ops._ext import require
  from xotorch_support_jetson_amd.ops.weights_layout import shuffle_for_stream
  torch.manual_seed(M + splits)
  N, Kd = 1024, 1280
  x = torch.randn(M, Kd, device=gpu, dtype=torch.bfloat16)
  w = torch.randn(N, Kd, device=gpu, dtype=torch.bfloat16) / math.sqrt(Kd)
  b = torch.randn(N, device=gpu, dtype=torch.bfloat16)
  r = torch.randn(M, N, device=gpu, dtype=torch.bfloat16)
  ws = torch.empty(splits * M * N, device=gpu, dtype=torch.float32)
  full = R.linear(x, w, b)
  if epi == "silu":
    f = full.view(M, N // 32, 2, 16)
    ref = (torch.nn.functional.silu(f[:, :, 0]) * f[:, :, 1]).reshape(M, N // 2)
    y = torch.empty(M, N // 2, device=gpu, dtype=torch.float32 if f32 else torch.bfloat16)
  elif epi == "resid":
    ref = full + r.float()
    y = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
  else:
    ref = full
    y = torch.empty(M, N, device=gpu, dtype=torch.float32 if f32 else torch.bfloat16)
  require().gemm_big(x, shuffle_for_stream(w), y, b, r if epi == "resid" else None, ws, K.EPI[epi], 4256, splits)
  assert rel_err(y, ref) < 1e-2


def test_gemm_w4_exact_layout(gpu):
  """Integer-valued operands: the four-wave tile matches bit for bit (fragment maps, the permuted weight rows and
  the XOR-4 weight image swizzle, the token-row swizzle, the shuffled k order), and in place with the residual."""
  from xotorch_support_jetson_amd.ops._ext import require
  from xotorch_support_jetson_amd.ops.weights_layout import shuffle_for_stream
  g = torch.Generator(device="cpu").manual_seed(6)
  M, N, Kd = 700, 768, 512
  x = torch.randint(-3, 4, (M, Kd), generator=g).to(torch.bfloat16).to(gpu)
  w = torch.randint(-3, 4, (N, Kd), generator=g).to(torch.bfloat16).to(gpu)
  ref = x.float() @ w.float().t()
  y = torch.zeros(M, N, device=gpu, dtype=torch.float32)
  require().gemm_big(x, shuffle_for_stream(w), y, None, None, None, 0, 4256, 1)
  assert torch.equal(y, ref)
  h = torch.randint(-3, 4, (M, N), generator=g).to(torch.bfloat16).to(gpu)
  want = (h.float() + ref).to(torch.bfloat16)
  require().gemm_big(x, shuffle_for_stream(w), h, None, h, None, 1, 4256, 1)
  assert torch.equal(h, want)


def test_gemm_big_exact_layout(gpu):
  """Integer-valued operands (exact in bf16 and fp32): every output element must match bit for bit,
  which pins the fragment maps, the LDS swizzle and the shuffled-layout k order."""
  from xotorch_support_jetson_amd.ops._ext import require
  from xotorch_support_jetson_amd.ops.weights_layout import shuffle_for_stream
  g = torch.Generator(device="cpu").manual_seed(5)
  M, N, Kd = 300, 512, 384
  x = torch.randint(-3, 4, (M, Kd), generator=g).to(torch.bfloat16).to(gpu)
  w = torch.randint(-3, 4, (N, Kd), generator=g).to(torch.bfloat16).to(gpu)
  y = torch.empty(M, N, device=gpu, dtype=torch.float32)
  ref = x.float() @ w.float().t()
  # 1256: ping-pong schedule of the 256 x 256 tile; 224: odd row groups per wave; + 10000 x BM: short row tiles
  for bn in (256, 128, 1256, 224, 2240256, 1600128, 1920256):
    y.zero_()
    require().gemm_big(x, shuffle_for_stream(w), y, None, None, None, 0, bn, 1)
    assert torch.equal(y, ref), bn


# ------------------------------------------------------------------ mixture of experts
@pytest.mark.parametrize("T,E,k,F", [(1, 8, 2, 512), (7, 8, 2, 512), (100, 8, 2, 512), (300, 4, 2, 512),
                                     (64, 16, 4, 512), (64, 16, 4, 384), (1, 8, 2, 384)])
@pytest.mark.parametrize("shuffled", [False, True])
def test_moe_layer(gpu, T, E, k, F, shuffled):
  """route -> grouped gate/up (gathered rows, SiLU*mul) -> grouped down -> combine, vs an fp32
  per-expert reference of the same Mixtral MoE block (F = 384: an odd count of 128-deep k-chunks in the
  down projection, as DeepSeek-V2-Lite's 1408)."""
  from xotorch_support_jetson_amd.ops._ext import require
  from xotorch_support_jetson_amd.ops.weights_layout import shuffle_for_stream
  torch.manual_seed(T + E)
  C = require()
  D = 256
  x = torch.randn(T, D, device=gpu).to(torch.bfloat16)
  h = torch.randn(T, D, device=gpu).to(torch.bfloat16)
  router = torch.randn(T, E, device=gpu, dtype=torch.float32)
  gu = (torch.randn(E, 2 * F, D, device=gpu) / math.sqrt(D)).to(torch.bfloat16)  # 16-row interleaved g/u
  down = (torch.randn(E, D, F, device=gpu) / math.sqrt(F)).to(torch.bfloat16)
  # fp32 reference
  probs = torch.softmax(router, -1)
  tw, ti = torch.topk(probs, k, -1)
  tw = tw / tw.sum(-1, keepdim=True)
  ref = h.float().clone()
  for t in range(T):
    for j in range(k):
      e = int(ti[t, j])
      g = (x[t].float() @ gu[e].float().t()).view(-1, 2, 16)
      a = torch.nn.functional.silu(g[:, 0]) * g[:, 1]
      ref[t] += tw[t, j] * (a.reshape(-1).to(torch.bfloat16).float() @ down[e].float().t())
  topw = torch.empty(T * k, device=gpu)
  topi = torch.empty(T * k, dtype=torch.int32, device=gpu)
  slot_of = torch.empty_like(topi)
  sorted_tok = torch.empty_like(topi)
  off = torch.empty(E + 1, dtype=torch.int32, device=gpu)
  C.moe_route(router, k, topw, topi, slot_of, sorted_tok, off)
  assert torch.equal(torch.sort(topi.view(T, k).long(), -1)[0], torch.sort(ti, -1)[0])
  assert int(off[-1]) == T * k and torch.equal(torch.sort(slot_of.long())[0], torch.arange(T * k, device=gpu))
  gw = torch.stack([shuffle_for_stream(gu[e]) for e in range(E)]) if shuffled else gu
  dw = torch.stack([shuffle_for_stream(down[e]) for e in range(E)]) if shuffled else down
  act = torch.empty(T * k, F, dtype=torch.bfloat16, device=gpu)
  C.gemm_moe(x, gw, act, off, sorted_tok, 2, T, shuffled)
  Ss = (1, 2) if F % 256 == 0 else (1, 3)
  for S in Ss:  # down projection whole, and split over K into fp32 slabs summed by the combine
    y = torch.empty(S * T * k, D, dtype=torch.float32, device=gpu)
    C.gemm_moe(act, dw, y, off, None, 0, T, shuffled, S)
    out = h.clone()
    C.moe_combine(y, slot_of, topw, out, S)
    assert rel_err(out.float() - h.float(), ref - h.float()) < 3e-2, S  # the MoE contribution itself
    # combine fused with the following RMSNorm: same residual stream, normed output == rmsnorm(stream)
    lnw = torch.randn(D, device=gpu).to(torch.bfloat16)
    h2, normed = h.clone(), torch.empty_like(h)
    C.moe_combine_norm(y, slot_of, topw, h2, S, lnw, normed, 1e-5)
    assert torch.equal(h2, out), S
    assert rel_err(normed, R.rmsnorm(out, lnw, 1e-5)[0]) < 1e-2, S
  if shuffled:  # the same block on gemm_big tiles (128-, 192- and 256-row tiles per expert)
    for bm in (128, 192, 256, 1128, 1192, 1256, 2256, 2192, 2128):  # + 1000: deeper LDS pipelines; 2xxx: two-phase
      act2 = torch.empty_like(act)
      C.gemm_moe(x, gw, act2, off, sorted_tok, 2, T, True, 1, bm)
      assert rel_err(act2, act) < 1e-2, bm
      for S in Ss:
        y = torch.empty(S * T * k, D, dtype=torch.float32, device=gpu)
        C.gemm_moe(act2, dw, y, off, None, 0, T, True, S, bm)
        out = h.clone()
        C.moe_combine(y, slot_of, topw, out, S)
        assert rel_err(out.float() - h.float(), ref - h.float()) < 3e-2, (bm, S)


@pytest.mark.parametrize("B,L,H,Hkv,Dh", [(1, 64, 4, 1, 64), (2, 100, 8, 2, 128), (1, 300, 8, 8, 64),
                                          (2, 257, 16, 4, 128), (1, 130, 4, 4, 192), (1, 1024, 8, 2, 128)])
def test_attention_train_fwd_bwd(gpu, B, L, H, Hkv, Dh):
  """Training attention kernels (fwd, dQ, dK/dV) vs fp32 torch autograd of causal GQA attention, with
  q / k / v given as strided row views of one fused qkv tensor (as the trainer passes them)."""
  from xotorch_support_jetson_amd.train import autograd_ops as A
  torch.manual_seed(L + H)
  qkv = (torch.randn(B * L, (H + 2 * Hkv) * Dh, device=gpu) * 0.5).to(torch.bfloat16).requires_grad_()
  q = qkv[:, :H * Dh]
  k = qkv[:, H * Dh:(H + Hkv) * Dh]
  v = qkv[:, (H + Hkv) * Dh:]
  o = A.attention(q, k, v, B, L, H, Hkv, Dh)
  do = torch.randn_like(o)
  o.backward(do)
  g = qkv.grad.float().clone()
  x = qkv.detach().float().requires_grad_()
  ref = A._attn_ref(x[:, :H * Dh], x[:, H * Dh:(H + Hkv) * Dh], x[:, (H + Hkv) * Dh:], B, L, H, Hkv, Dh)
  ref.backward(do.float())
  assert rel_err(o, ref) < 2e-2
  for name, sl in (("dq", slice(0, H * Dh)), ("dk", slice(H * Dh, (H + Hkv) * Dh)), ("dv", slice((H + Hkv) * Dh, None))):
    assert rel_err(g[:, sl], x.grad[:, sl]) < 3e-2, name


@pytest.mark.parametrize("B,L,H,Hkv,Dh", [(2, 100, 8, 2, 128), (1, 257, 16, 4, 128), (1, 130, 4, 4, 64)])
def test_qkv_attention_fused_matches_separate(gpu, B, L, H, Hkv, Dh):
  """QKVAttentionFn (one rope launch for q and k, dv straight into dqkv) against QKVRopeFn + AttentionFn: the same
  kernels on the same values, so output and dqkv are bitwise equal."""
  from xotorch_support_jetson_amd.train import autograd_ops as A
  torch.manual_seed(L)
  ang = torch.rand(512, Dh // 2, device=gpu) * 6.28  # any table: both paths rotate with the same one
  cos_sin = torch.cat([ang.cos(), ang.sin()], 1).contiguous()
  pos = (torch.arange(L, device=gpu, dtype=torch.int32)).repeat(B)
  W = (H + 2 * Hkv) * Dh
  x = (torch.randn(B * L, W, device=gpu) * 0.5).to(torch.bfloat16)
  do = torch.randn(B * L, H * Dh, device=gpu).to(torch.bfloat16)
  a = x.clone().requires_grad_()
  oa = A.qkv_attention(a, pos, cos_sin, B, L, H, Hkv, Dh)
  oa.backward(do)
  b = x.clone().requires_grad_()
  q, k, v = A.qkv_rope(b, pos, cos_sin, H, Hkv, Dh)
  ob = A.attention(q, k, v, B, L, H, Hkv, Dh)
  ob.backward(do)
  assert torch.equal(oa, ob)
  assert torch.equal(a.grad, b.grad)


@pytest.mark.parametrize("B,L,H", [(1, 100, 4), (2, 300, 8)])
def test_attention_qk_v_deepseek_dims(gpu, B, L, H):
  """DeepSeek MLA training attention (q / k heads of 192, v heads of 128, v zero-padded to 192 for the 192-wide
  kernel, custom softmax scale) vs fp32 SDPA autograd: output and all three input gradients."""
  import torch.nn.functional as F
  from xotorch_support_jetson_amd.train import autograd_ops as A
  torch.manual_seed(L + H)
  T, dqk, dv, scale = B * L, 192, 128, 0.1
  q, k = ((torch.randn(T, H * dqk, device=gpu) * 0.5).to(torch.bfloat16).requires_grad_() for _ in range(2))
  v = (torch.randn(T, H * dv, device=gpu) * 0.5).to(torch.bfloat16).requires_grad_()
  o = A.attention_qk_v(q, k, v, B, L, H, dqk, dv, scale)
  do = torch.randn_like(o)
  o.backward(do)
  xs = [t.detach().float().requires_grad_() for t in (q, k, v)]
  hd = lambda t: t.reshape(B, L, H, -1).transpose(1, 2)
  ref = F.scaled_dot_product_attention(hd(xs[0]), hd(xs[1]), hd(xs[2]), is_causal=True, scale=scale)
  ref = ref.transpose(1, 2).reshape(T, H * dv)
  ref.backward(do.float())
  assert rel_err(o, ref) < 2e-2
  for name, t, x in zip("qkv", (q, k, v), xs):
    assert rel_err(t.grad, x.grad) < 3e-2, name


@pytest.mark.parametrize("B,L,H,Dh", [(1, 577, 16, 64), (2, 64, 4, 128), (3, 100, 8, 64), (1, 1, 2, 128)])
def test_attention_bidir(gpu, B, L, H, Dh):
  """Bidirectional attention (the vision tower's) on the training forward kernel with the causal mask off vs
  fp32 softmax(q k^T) v, q / k / v as column slices of one qkv tensor."""
  torch.manual_seed(B * L + H)
  qkv = (torch.randn(B * L, 3 * H * Dh, device=gpu) * 0.5).to(torch.bfloat16)
  q, k, v = qkv[:, :H * Dh], qkv[:, H * Dh:2 * H * Dh], qkv[:, 2 * H * Dh:]
  got = K.attention_bidir(q, k, v, B, L, H, Dh, Dh ** -0.5)
  ref = K.attention_bidir(*(t.float().cpu() for t in (q, k, v)), B, L, H, Dh, Dh ** -0.5)
  assert rel_err(got.cpu(), ref) < 2e-2


def test_vision_tower_gpu_matches_cpu(gpu):
  """CLIP-L-shaped tower (1024 wide, 16 heads of 64, 336 px: 577 tokens; one layer run) + projector on the GPU
  path -- weights shuffled into the stream layout (patch embedding K padded 588 -> 640), attention on the MFMA
  kernel -- vs the fp32 CPU path on the same weights."""
  import dataclasses
  from xotorch_support_jetson_amd.models.config import preset
  from xotorch_support_jetson_amd.models.vision import image_features, random_vision
  c = preset("llava-1.5-7b-hf")
  c = dataclasses.replace(c, vision=dict(c.vision, num_hidden_layers=2))
  vw = random_vision(c, "cpu", seed=4)
  pixels = torch.randn(2, 3, 336, 336, generator=torch.Generator().manual_seed(2))
  ref = image_features(c, vw, pixels)
  vg = {k: t.to(gpu) for k, t in vw.items()}
  got = image_features(c, vg, pixels.to(gpu))
  assert got.shape == ref.shape == (2 * 576, c.hidden_size)
  assert rel_err(got.cpu(), ref) < 3e-2
  # a second image on the same weights dict reuses the shuffled copies (identity-keyed cache)
  again = image_features(c, vg, pixels[:1].to(gpu))
  assert rel_err(again.cpu(), ref[:576]) < 3e-2


@pytest.mark.parametrize("T,E,D", [(1, 8, 4096), (37, 8, 4096), (512, 8, 1024), (5, 4, 256), (9, 16, 512),
                                   (1, 64, 2048), (37, 64, 2048), (4099, 64, 2048), (300, 160, 5120), (17, 256, 7168),
                                   (3, 32, 512), (40, 128, 4096), (16, 160, 5120)])
def test_router_logits(gpu, T, E, D):
  from xotorch_support_jetson_amd.ops._ext import require
  torch.manual_seed(0)
  x = torch.randn(T, D, device=gpu, dtype=torch.bfloat16)
  w = (torch.randn(E, D, device=gpu) * 0.05).to(torch.bfloat16)
  out = torch.empty(T, E, device=gpu, dtype=torch.float32)
  require().router_logits(x, w, out)
  ref = x.float() @ w.float().t()
  assert rel_err(out, ref) < 1e-5


@pytest.mark.parametrize("T", [1, 5])
@pytest.mark.parametrize("shuffled", [False, True])
def test_moe_gate_up_split_k(gpu, T, shuffled):
  """Decode-sized MoE batches: grouped gate/up split over K into fp32 slabs + SiLU slab reduce == the
  fused SiLU-epilogue grouped GEMM."""
  from xotorch_support_jetson_amd.ops._ext import require
  from xotorch_support_jetson_amd.ops.weights_layout import shuffle_for_stream
  torch.manual_seed(T)
  C = require()
  E, k, D, F, S = 8, 2, 1024, 512, 4
  x = torch.randn(T, D, device=gpu).to(torch.bfloat16)
  gu = (torch.randn(E, 2 * F, D, device=gpu) / math.sqrt(D)).to(torch.bfloat16)
  gw = torch.stack([shuffle_for_stream(gu[e]) for e in range(E)]) if shuffled else gu
  topw = torch.empty(T * k, device=gpu)
  topi = torch.empty(T * k, dtype=torch.int32, device=gpu)
  slot_of, sorted_tok = torch.empty_like(topi), torch.empty_like(topi)
  off = torch.empty(E + 1, dtype=torch.int32, device=gpu)
  C.moe_route(torch.randn(T, E, device=gpu), k, topw, topi, slot_of, sorted_tok, off)
  act = torch.empty(T * k, F, dtype=torch.bfloat16, device=gpu)
  C.gemm_moe(x, gw, act, off, sorted_tok, 2, T, shuffled)
  ys = torch.empty(S * T * k, 2 * F, dtype=torch.float32, device=gpu)
  C.gemm_moe(x, gw, ys, off, sorted_tok, 0, T, shuffled, S)
  act2 = torch.empty_like(act)
  C.splitk_silu(ys, S, act2)
  assert rel_err(act2, act) < 1e-2


# ---------------------------------------------------------------------------- DeepSeek MLA / routing
def _mla_cache(num_pages, DL, DR, dev, seed=0):
  g = torch.Generator(device=dev).manual_seed(seed)
  return torch.randn(num_pages, 64, DL + DR, device=dev, dtype=torch.bfloat16, generator=g)


@pytest.mark.parametrize("wide", ["0", "1"])
@pytest.mark.parametrize("DL", [512, 256])
@pytest.mark.parametrize("H", [16, 4, 40, 128, 200])
@pytest.mark.parametrize("ctxs", [[1, 64, 65, 300], [1000]])
def test_mla_attn_decode(gpu, DL, H, ctxs, wide, monkeypatch):
  """Narrow (16 heads per workgroup) and many-head (up to 128 heads per workgroup, 1 to 8 waves, several
  head groups past 128) kernels, one partition and split-KV + combine."""
  monkeypatch.setenv("XOT_MLA_WIDE", wide)
  torch.manual_seed(0)
  DR, B = 64, len(ctxs)
  width = max(-(-c // 64) for c in ctxs)
  num_pages = B * width + 3
  cache = _mla_cache(num_pages, DL, DR, gpu)
  perm = torch.randperm(num_pages - 3)[:B * width].view(B, width).int()
  bt = perm.to(gpu)
  ctx = torch.tensor(ctxs, dtype=torch.int32, device=gpu)
  cu = torch.arange(B + 1, dtype=torch.int32, device=gpu)
  q_lat = torch.randn(H, B, DL, device=gpu, dtype=torch.bfloat16)
  q_pe = torch.randn(B, H * DR + 8, device=gpu, dtype=torch.bfloat16)[:, :H * DR]  # strided rows
  scale = 0.1
  ref = R.mla_attn(q_lat.cpu(), q_pe.cpu(), cache.cpu(), bt.cpu(), cu.cpu(), ctx.cpu(), scale)
  for ws in (None, K.MLAWorkspace(B, H, DL, width * 64, gpu)):  # one partition / split-KV + combine
    out = K.mla_attn(q_lat, q_pe, cache, bt, cu, ctx, scale, ws)
    assert rel_err(out.cpu(), ref) < 2e-2, (DL, H, ctxs)


@pytest.mark.parametrize("wide,H", [("0", 16), ("1", 16), ("1", 128)])
@pytest.mark.parametrize("DL", [512, 256])
def test_mla_attn_prefill_causal(gpu, DL, wide, H, monkeypatch):
  monkeypatch.setenv("XOT_MLA_WIDE", wide)
  torch.manual_seed(1)
  DR = 64
  qlens, ctxs = [37, 1, 130], [37, 70, 200]  # second / third: chunked prefill on top of a cached prefix
  B = len(qlens)
  width = max(-(-c // 64) for c in ctxs)
  cache = _mla_cache(B * width + 1, DL, DR, gpu, seed=1)
  bt = torch.arange(B * width, dtype=torch.int32, device=gpu).view(B, width)
  cu = torch.tensor([0] + list(torch.tensor(qlens).cumsum(0)), dtype=torch.int32, device=gpu)
  T = int(cu[-1])
  ctx = torch.tensor(ctxs, dtype=torch.int32, device=gpu)
  q_lat = torch.randn(H, T, DL, device=gpu, dtype=torch.bfloat16)
  q_pe = torch.randn(T, H * DR, device=gpu, dtype=torch.bfloat16)
  ref = R.mla_attn(q_lat.cpu(), q_pe.cpu(), cache.cpu(), bt.cpu(), cu.cpu(), ctx.cpu(), 0.08)
  out = K.mla_attn(q_lat, q_pe, cache, bt, cu, ctx, 0.08, K.MLAWorkspace(T, H, DL, width * 64, gpu))
  assert rel_err(out.cpu(), ref) < 2e-2


def test_mla_prep(gpu):
  torch.manual_seed(2)
  T, H, DL, DR = 9, 16, 512, 64
  ckv_full = torch.randn(T, 128 + DL + DR, device=gpu, dtype=torch.bfloat16)
  ckv = ckv_full[:, 128:]  # strided rows, as sliced out of the fused A projection
  kv_ln = torch.randn(DL, device=gpu, dtype=torch.bfloat16)
  q = torch.randn(T, H * 192, device=gpu, dtype=torch.bfloat16)
  pos = torch.arange(5, 5 + T, dtype=torch.int32, device=gpu)
  cs = build_cos_sin(DR, 64, 10000.0, None, device=gpu)
  slots = torch.tensor([3, 70, -1, 5, 6, 7, 8, 9, 100], dtype=torch.int64, device=gpu)
  cache = torch.zeros(4, 64, DL + DR, device=gpu, dtype=torch.bfloat16)
  q2, cache2 = q.clone().cpu(), cache.clone().cpu()
  K.mla_prep(ckv, kv_ln, q, H * 128, H, pos, cs, slots, cache, 1e-6)
  R.mla_prep(ckv.cpu(), kv_ln.cpu(), q2, H * 128, H, pos.cpu(), cs.cpu(), slots.cpu(), cache2, 1e-6)
  assert rel_err(q.cpu(), q2) < 1e-2
  assert rel_err(cache.cpu(), cache2) < 1e-2


@pytest.mark.parametrize("E,k,ng,tg,method,sig,norm", [(64, 6, 1, 1, 0, False, False), (8, 2, 4, 2, 1, False, False),
                                                        (256, 8, 8, 4, 2, True, True), (16, 4, 4, 2, 2, True, True)])
def test_moe_route_ds(gpu, E, k, ng, tg, method, sig, norm):
  torch.manual_seed(3)
  T = 300
  logits = torch.randn(T, E, device=gpu) * 2
  bias = torch.randn(E, device=gpu) * 0.05 if sig else None
  topw, topi, slot_of, sorted_tok, off = K.moe_route_ds(logits, bias, k, ng, tg, method, sig, norm, 2.5)
  rw, ri = R.moe_route_ds(logits.cpu(), bias.cpu() if bias is not None else None, k, ng, tg, method, sig, norm, 2.5)
  got_i, order = topi.view(T, k).cpu().long().sort(-1)
  exp_i, eorder = ri.sort(-1)
  assert torch.equal(got_i, exp_i)
  torch.testing.assert_close(topw.view(T, k).cpu().gather(1, order), rw.gather(1, eorder), rtol=1e-4, atol=1e-5)
  # slot bookkeeping: every (token, j) slot points back at its token inside its expert's range
  off_c, st = off.cpu(), sorted_tok.cpu()
  so = slot_of.view(T, k).cpu()
  for t in range(0, T, 37):
    for j in range(k):
      e = int(topi.view(T, k)[t, j])
      assert off_c[e] <= so[t, j] < off_c[e + 1] and int(st[so[t, j]]) == t


@pytest.mark.parametrize("R,C", [(256, 384), (128, 64), (512, 1024), (384, 1152), (1280, 256)])
def test_relayout_kernels(gpu, R, C):
  """csrc/layout.hip: shuffle / shuffle of the transpose / transpose vs the torch permutations, from a
  row-strided source, into a pre-filled destination (every element written)."""
  from xotorch_support_jetson_amd.ops._ext import require
  from xotorch_support_jetson_amd.ops.weights_layout import shuffle_for_stream
  from xotorch_support_jetson_amd.train.autograd_ops import relayout
  torch.manual_seed(0)
  big = torch.randn(R, C + 64, device=gpu, dtype=torch.bfloat16)
  src = big[:, :C]
  if C % 128 == 0:
    assert torch.equal(relayout(src, 0), shuffle_for_stream(src.contiguous()))
  assert torch.equal(relayout(src, 1), shuffle_for_stream(src.t().contiguous()))
  assert torch.equal(relayout(src, 2), src.t().contiguous())
  for mode, want in ((1, shuffle_for_stream(src.t().contiguous())), (2, src.t().contiguous())):
    out = torch.full((C * R,), 7.0, device=gpu, dtype=torch.bfloat16).view(want.shape)
    require().relayout(src, out, mode)
    assert torch.equal(out, want), mode


@pytest.mark.parametrize("T,M,N", [(64, 256, 256), (192, 512, 768), (4096, 256, 512)])
@pytest.mark.parametrize("resid", [False, True])
def test_gemm_tn(gpu, T, M, N, resid):
  """csrc/gemm_w4.hip TN (the weight-gradient GEMM on token-major operands, fragments read transposed out of LDS):
  y (+)= dy^T . x from a row-strided dy, against fp32 torch."""
  from xotorch_support_jetson_amd.ops._ext import require
  torch.manual_seed(T + M)
  dy = (torch.randn(T, M + 64, device=gpu) * 0.5).to(torch.bfloat16)[:, :M]
  x = torch.randn(T, N, device=gpu).to(torch.bfloat16)
  y0 = (torch.randn(M, N, device=gpu) * 4).to(torch.bfloat16)
  y = y0.clone()
  require().gemm_tn(dy, x, y, resid)
  want = dy.float().t() @ x.float() + (y0.float() if resid else 0.0)
  err = ((y.float() - want).norm() / want.norm()).item()
  assert err < 5e-3, err
  if not resid:  # fp32 output
    y32 = torch.empty(M, N, device=gpu)
    require().gemm_tn(dy, x, y32, False)
    assert ((y32 - dy.float().t() @ x.float()).norm() / want.norm()).item() < 1e-4


def test_gemm_tn_exact_layout(gpu):
  """Integer operands (exact in bf16 and fp32): every element of dy^T . x bit-exact, so a wrong swizzle, fragment
  order or tile mapping cannot hide in the tolerance."""
  from xotorch_support_jetson_amd.ops._ext import require
  g = torch.Generator(device=gpu).manual_seed(1)
  T, M, N = 128, 512, 768
  dy = torch.randint(-1, 2, (T, M), device=gpu, generator=g).to(torch.bfloat16)
  x = torch.randint(-1, 2, (T, N), device=gpu, generator=g).to(torch.bfloat16)
  y = torch.full((M, N), 3.0, device=gpu, dtype=torch.bfloat16)
  require().gemm_tn(dy, x, y, True)
  assert torch.equal(y.float(), dy.float().t() @ x.float() + 3.0)


def test_dw_tn_ragged_tokens(gpu, monkeypatch):
  """train/autograd_ops.dw_tn pads a ragged token count (37) with zero rows; the result equals the fp32 product."""
  from xotorch_support_jetson_amd.train import autograd_ops as A
  from xotorch_support_jetson_amd.train.autograd_ops import dw_tn
  monkeypatch.setattr(A, "DW_TN", True)
  torch.manual_seed(0)
  dy = torch.randn(37, 256, device=gpu).to(torch.bfloat16)
  x = torch.randn(37, 512, device=gpu).to(torch.bfloat16)
  out = torch.empty(256, 512, device=gpu, dtype=torch.bfloat16)
  assert dw_tn(dy, x, out, False)
  want = dy.float().t() @ x.float()
  assert ((out.float() - want).norm() / want.norm()).item() < 5e-3


@pytest.mark.parametrize("with_h", [False, True])
@pytest.mark.parametrize("T,Kd,N", [(256, 384, 512), (192, 512, 768)])
def test_own_linear_grads_match_torch(gpu, with_h, T, Kd, N):
  """OwnLinearFn (forward, dX, dW accumulated over two micro-batches into the GradAcc buffer) on the MFMA
  GEMMs vs fp32 torch autograd."""
  from xotorch_support_jetson_amd.train import autograd_ops as A
  torch.manual_seed(0)
  w = (torch.randn(N, Kd, device=gpu) / math.sqrt(Kd)).to(torch.bfloat16).requires_grad_(True)
  tw, acc = A.TrainWeight(w), A.GradAcc("w", w)
  assert tw.ok
  xs = [torch.randn(T, Kd, device=gpu, dtype=torch.bfloat16) for _ in range(2)]
  hs = [torch.randn(T, N, device=gpu, dtype=torch.bfloat16) for _ in range(2)]
  gs = [torch.randn(T, N, device=gpu, dtype=torch.bfloat16) for _ in range(2)]
  dw_ref = torch.zeros(N, Kd, device=gpu)
  for x, h, g in zip(xs, hs, gs):
    xl = x.clone().requires_grad_(True)
    y = A.linear_own(xl, w, tw, acc, h if with_h else None)
    yr = x.float() @ w.detach().float().t() + (h.float() if with_h else 0)
    assert rel_err(y, yr) < 1e-2
    y.backward(g)
    assert rel_err(xl.grad, g.float() @ w.detach().float()) < 1e-2
    dw_ref += g.float().t() @ x.float()
  assert w.grad is None
  assert rel_err(acc.buf, dw_ref) < 1e-2


@pytest.mark.parametrize("resid", [False, True])
def test_gemm_kgroup(gpu, resid):
  """K-grouped GEMM (grouped experts' weight gradients): y[e] (+)= x[:, koff[e]:koff[e+1]] . w[:, ...]^T with
  64-aligned segments, an empty one included, vs fp32 torch per segment."""
  from xotorch_support_jetson_amd.ops._ext import require
  from xotorch_support_jetson_amd.ops.weights_layout import shuffle_for_stream
  torch.manual_seed(0)
  M, N = 320, 272
  segs = [128, 0, 64, 384, 64]
  K = sum(segs)
  koff = torch.tensor([0] + list(torch.tensor(segs).cumsum(0)), dtype=torch.int32, device=gpu)
  x = torch.randn(M, K, device=gpu, dtype=torch.bfloat16)
  w = torch.randn(N, K, device=gpu, dtype=torch.bfloat16) / 8
  y0 = torch.randn(len(segs), M, N, device=gpu, dtype=torch.bfloat16)
  y = y0.clone()
  require().gemm_kgroup(x, shuffle_for_stream(w), y, koff, resid)
  for e in range(len(segs)):
    a, b = int(koff[e]), int(koff[e + 1])
    ref = x[:, a:b].float() @ w[:, a:b].float().t() + (y0[e].float() if resid else 0)
    assert rel_err(y[e], ref) < 1e-2 if ref.norm() > 0 else y[e].abs().max() == 0


# ------------------------------------------------------------------ stream-K GEMM (the headline's gate/up)
@pytest.mark.parametrize("rows,D,S", [(1, 8192, 4), (300, 8192, 4), (512, 8192, 4), (512, 8192, 3), (512, 4096, 4),
                                      (256, 5120, 2), (512, 8192, 5)])
def test_splitk_resid_rmsnorm(gpu, rows, D, S):
  """Split-K slab reduce + bias + residual (in place) + RMSNorm vs fp32: the 256-thread rows and the 1024-thread
  wide rows (D = 8192 at 256+ rows), unrolled and runtime slab counts."""
  from xotorch_support_jetson_amd.ops._ext import require
  torch.manual_seed(rows + D + S)
  ws = torch.randn(S * rows * D, device=gpu, dtype=torch.float32)
  h = torch.randn(rows, D, device=gpu, dtype=torch.bfloat16)
  bias = torch.randn(D, device=gpu, dtype=torch.bfloat16)
  w = (1 + 0.1 * torch.randn(D, device=gpu)).to(torch.bfloat16)
  out = torch.empty(rows, D, device=gpu, dtype=torch.bfloat16)
  ref_h = (h.float() + bias.float() + ws.view(S, rows, D).sum(0)).to(torch.bfloat16)
  hf = ref_h.float()
  ref = hf * torch.rsqrt(hf.pow(2).mean(-1, keepdim=True) + 1e-5) * w.float()
  require().splitk_resid_rmsnorm(ws, S, bias, h, w, out, 1e-5)
  assert rel_err(h, ref_h) < 1e-2
  assert rel_err(out, ref) < 1e-2

"""Plain-PyTorch fp32 implementations of every kernel in the library.

These are (1) the numerical oracles the HIP kernels are tested against and (2) the compute path on
CPU-only hosts (BASELINE config 1: Llama-3.2-1B on the CPU engine).  Semantics match the kernels
exactly, including the paged KV layout (K [pages, Hkv, 64, Dh], V [pages, Hkv, Dh, 64] storage holding each page
chunk-major, see v_chunks).
"""
from __future__ import annotations

import os
import weakref

import torch
import torch.nn.functional as F

PAGE = 64


def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float, residual: torch.Tensor | None = None):
  """Returns (normed, new_residual). new_residual = bf16(x + residual) when residual is given."""
  if residual is not None:
    x = (x.float() + residual.float()).to(x.dtype)
  xf = x.float()
  y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * w.float()
  return y.to(x.dtype), (x if residual is not None else None)


def rope(x: torch.Tensor, pos: torch.Tensor, cos_sin: torch.Tensor, inverse: bool = False) -> torch.Tensor:
  """x [T, nh, Dh]; HF rotate-half convention."""
  Dh = x.shape[-1]
  half = Dh // 2
  cs = cos_sin[pos.long()].to(x.device)  # [T, Dh]
  cos, sin = cs[:, None, :half], cs[:, None, half:]
  if inverse:
    sin = -sin
  xf = x.float()
  x0, x1 = xf[..., :half], xf[..., half:]
  return torch.cat([x0 * cos - x1 * sin, x1 * cos + x0 * sin], dim=-1).to(x.dtype)


def silu_mul(gu: torch.Tensor) -> torch.Tensor:
  Fd = gu.shape[-1] // 2
  g, u = gu[..., :Fd].float(), gu[..., Fd:].float()
  return (F.silu(g) * u).to(gu.dtype)


# fp32 copies of low-precision CPU weights, made once per tensor and re-made when the tensor is written in place
# (its version counter moves) or re-pointed: without them every CPU token widened every weight again (~1 s per
# token for Llama-3.2-1B).  Tensors that require grad (trained parameters) are widened per call as before.
# at most this many bytes of fp32 copies live at once (XOT_CPU_F32_CACHE_GB): a model too large for it widens the
# rest per call, as before
_F32_BUDGET = int(float(os.environ.get("XOT_CPU_F32_CACHE_GB", "12")) * (1 << 30))
_f32_bytes = [0]


def _release(n: int) -> None:
  _f32_bytes[0] -= n


def _wide(w: torch.Tensor) -> torch.Tensor:
  if w.dtype == torch.float32 or w.device.type != "cpu" or w.requires_grad or w.grad_fn is not None:
    return w.float()
  key = (w._version, w.data_ptr(), tuple(w.shape), tuple(w.stride()))
  got = getattr(w, "_xot_f32", None)  # kept on the tensor: freed with it
  if got is not None and got[0] == key:
    return got[1]
  f = w.float()
  n = f.numel() * 4
  if got is None and _f32_bytes[0] + n > _F32_BUDGET:
    return f
  if got is None:
    _f32_bytes[0] += n
    weakref.finalize(w, _release, n)
  w._xot_f32 = (key, f)
  return f


def linear(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor | None = None) -> torch.Tensor:
  y = x.float() @ _wide(w).t()
  if bias is not None:
    y = y + bias.float()
  return y


def v_chunks(v_cache: torch.Tensor) -> torch.Tensor:
  """The V pool [pages, Hkv, Dh, BS] (storage shape) as the layout the kernels use: each page of a KV head
  chunk-major, [BS / 8 chunks][Dh][8 keys] (csrc/common.h v_page_off)."""
  nb, Hkv, Dh, BS = v_cache.shape
  return v_cache.view(nb, Hkv, BS // 8, Dh, 8)


def write_kv(k: torch.Tensor, v: torch.Tensor, slots: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor):
  """k, v [T, Hkv, Dh] -> paged caches at global slots (slot < 0 skipped)."""
  BS = k_cache.shape[2]
  ok = slots >= 0
  s = slots[ok].long()
  blk, off = s // BS, s % BS
  k_cache[blk, :, off, :] = k[ok].to(k_cache.dtype)
  v_chunks(v_cache)[blk, :, off // 8, :, off % 8] = v[ok].to(v_cache.dtype)


def gather_kv(k_cache, v_cache, table, n):
  """Dense [n, Hkv, Dh] K and V for one sequence from its block table."""
  BS = k_cache.shape[2]
  npg = (n + BS - 1) // BS
  pages = table[:npg].long()
  k = k_cache[pages].permute(0, 2, 1, 3).reshape(npg * BS, k_cache.shape[1], k_cache.shape[3])[:n]
  v = v_chunks(v_cache)[pages].permute(0, 2, 4, 1, 3).reshape(npg * BS, v_cache.shape[1], v_cache.shape[2])[:n]
  return k, v


def _attend(q, k, v, scale, causal_offset: int | None):
  # q [S, H, Dh], k/v [T, Hkv, Dh]
  H, Hkv = q.shape[1], k.shape[1]
  G = H // Hkv
  kf = k.float().repeat_interleave(G, dim=1)
  vf = v.float().repeat_interleave(G, dim=1)
  s = torch.einsum("shd,thd->hst", q.float(), kf) * scale
  if causal_offset is not None:
    S, T = q.shape[0], k.shape[0]
    qpos = torch.arange(S, device=q.device)[:, None] + causal_offset
    kpos = torch.arange(T, device=q.device)[None, :]
    s = s.masked_fill(kpos > qpos, float("-inf"))
  p = torch.softmax(s, dim=-1)
  return torch.einsum("hst,thd->shd", p, vf)


def attn_decode(q, k_cache, v_cache, block_tables, ctx_lens, scale):
  """q [B, H, Dh] -> [B, H, Dh]"""
  out = torch.empty_like(q)
  for b in range(q.shape[0]):
    n = int(ctx_lens[b])
    if n <= 0:
      out[b] = 0
      continue
    k, v = gather_kv(k_cache, v_cache, block_tables[b], n)
    out[b] = _attend(q[b:b + 1], k, v, scale, None)[0].to(q.dtype)
  return out


def attn_prefill(q, k_cache, v_cache, block_tables, cu_q, ctx_lens, scale):
  """q [T, H, Dh] (new tokens of all sequences) -> [T, H, Dh]; causal against the cached context."""
  out = torch.empty_like(q)
  for b in range(ctx_lens.numel()):
    q0, q1 = int(cu_q[b]), int(cu_q[b + 1])
    if q1 <= q0:
      continue
    n = int(ctx_lens[b])
    k, v = gather_kv(k_cache, v_cache, block_tables[b], n)
    out[q0:q1] = _attend(q[q0:q1], k, v, scale, n - (q1 - q0)).to(q.dtype)
  return out


def sample_greedy(logits: torch.Tensor) -> torch.Tensor:
  return logits.float().argmax(dim=-1).to(torch.int32)


def topk_mask(logits: torch.Tensor, k: int) -> torch.Tensor:
  """Boolean mask of entries >= the k-th largest value (ties kept), per row."""
  kth = torch.topk(logits.float(), k, dim=-1).values[:, -1:]
  return logits.float() >= kth


def cross_entropy(logits: torch.Tensor, targets: torch.Tensor):
  """Per-row loss (0 where target < 0) and lse."""
  lf = logits.float()
  lse = torch.logsumexp(lf, dim=-1)
  valid = targets >= 0
  tgt = targets.clamp(min=0).long()
  picked = lf.gather(1, tgt[:, None])[:, 0]
  loss = torch.where(valid, lse - picked, torch.zeros_like(lse))
  return loss, lse


# ------------------------------------------------------------------ DeepSeek MLA / MoE routing
def mla_prep(ckv, kv_ln, q, qpe_off: int, H: int, pos, cos_sin, slots, cache, eps: float):
  """Latent rmsnorm (HF DeepseekV2RMSNorm rounding: normalise, cast, times weight) + rope of the shared
  key -> cache[slot] = [c | k_pe]; q_pe of every head rotated in place.  cache [pages, 64, DL + DR]."""
  DL = kv_ln.numel()
  DR = cos_sin.shape[1]
  T = ckv.shape[0]
  x = ckv[:, :DL].float()
  c = (x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + eps)).to(ckv.dtype).float() * kv_ln.float()
  kpe = rope(ckv[:, DL:DL + DR].reshape(T, 1, DR), pos, cos_sin)[:, 0]
  qpe = q[:, qpe_off:qpe_off + H * DR].reshape(T, H, DR)
  q[:, qpe_off:qpe_off + H * DR] = rope(qpe, pos, cos_sin).reshape(T, H * DR)
  ok = slots >= 0
  flat = cache.view(-1, cache.shape[-1])
  row = torch.cat([c.to(cache.dtype), kpe.to(cache.dtype)], 1)
  flat[slots[ok].long()] = row[ok]


def mla_attn(q_lat, q_pe, cache, block_tables, cu_q, ctx_lens, scale: float):
  """q_lat [H, T, DL], q_pe [T, >= H*DR] -> o_lat [H, T, DL]: causal multi-query attention over the latent."""
  H, T, DL = q_lat.shape
  DR = cache.shape[-1] - DL
  out = torch.zeros_like(q_lat)
  for b in range(ctx_lens.numel()):
    q0, q1 = int(cu_q[b]), int(cu_q[b + 1])
    n = int(ctx_lens[b])
    if q1 <= q0 or n <= 0:
      continue
    npg = -(-n // PAGE)
    lat = cache[block_tables[b, :npg].long()].reshape(npg * PAGE, -1)[:n].float()  # [n, DL + DR]
    qf = torch.cat([q_lat[:, q0:q1].float(), q_pe[q0:q1, :H * DR].reshape(q1 - q0, H, DR).permute(1, 0, 2).float()], 2)
    s = torch.einsum("hsd,td->hst", qf, lat) * scale
    qpos = torch.arange(q1 - q0)[:, None] + (n - (q1 - q0))
    s = s.masked_fill(torch.arange(n)[None, :] > qpos, float("-inf"))
    p = torch.softmax(s, -1)
    out[:, q0:q1] = torch.einsum("hst,td->hsd", p, lat[:, :DL]).to(out.dtype)
  return out


def moe_route_ds(logits, bias, k: int, n_group: int, topk_group: int, method: int, sigmoid: bool, norm: bool,
                 scale: float):
  """HF DeepseekV2TopkRouter / DeepseekV3TopkRouter -> (topw [T, k], topi [T, k])."""
  lf = logits.float()
  scores = torch.sigmoid(lf) if sigmoid else torch.softmax(lf, -1)
  choice = scores + bias.float() if bias is not None else scores
  T, E = lf.shape
  if n_group > 1 and topk_group < n_group:
    g = choice.view(T, n_group, E // n_group)
    gs = g.topk(2, -1).values.sum(-1) if method == 2 else g.max(-1).values
    keep = torch.zeros_like(gs).scatter_(1, gs.topk(topk_group, -1).indices, 1.0)
    mask = keep[:, :, None].expand(T, n_group, E // n_group).reshape(T, E).bool()
    choice = choice.masked_fill(~mask, float("-inf"))
  topi = choice.topk(k, -1).indices
  topw = scores.gather(1, topi)
  if norm:
    topw = topw / (topw.sum(-1, keepdim=True) + 1e-20)
  return topw * scale, topi

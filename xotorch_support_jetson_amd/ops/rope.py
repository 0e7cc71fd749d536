"""Rotary-embedding tables (host-built once per model, consumed by the RoPE kernels).

Supports plain RoPE (Qwen2/Mistral/Llama-3 without scaling), Llama-3.1/3.2 "llama3" frequency
scaling, linear scaling and Phi-3 LongRoPE with partial rotary dims.  The reference picks torchtune
RoPE classes by model-id substring and reads the wrong config key ("rope_factor") for Llama scaling
(xotorch/inference/torch/models/general_mha.py:33-63, llm_utils.py:68-69); here the HF `rope_scaling`
dict is honoured as written and a missing dict means no scaling (so Llama-3-8B/70B build; the reference
KeyErrors on them).

Partial rotary (Phi-3: the first R = 0.75 Dh dims of a head rotate as pairs (j, j + R/2), the rest pass
through) needs no kernel variant: the q / k projection rows of every head are permuted at load time
(`rope_perm`) so that HF dim pairs (j, j + R/2) land on the kernels' pairs (p, p + Dh/2), and the table
holds cos = 1, sin = 0 on the pass-through pairs.  q . k is invariant under the same permutation of both,
V is untouched, so attention outputs are exactly HF's; checkpoints are written back in HF order.
"""
from __future__ import annotations

import math
from typing import Optional

import torch


def inv_frequencies(head_dim: int, theta: float, scaling: dict | None) -> torch.Tensor:
  inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
  if not scaling:
    return inv
  kind = scaling.get("rope_type", scaling.get("type", "default"))
  if kind == "llama3":
    factor = float(scaling.get("factor", 8.0))
    lo = float(scaling.get("low_freq_factor", 1.0))
    hi = float(scaling.get("high_freq_factor", 4.0))
    old = float(scaling.get("original_max_position_embeddings", 8192))
    lo_wl, hi_wl = old / lo, old / hi
    wl = 2 * math.pi / inv
    scaled = torch.where(wl > lo_wl, inv / factor, inv)
    smooth = (old / wl - lo) / (hi - lo)
    smoothed = (1 - smooth) * scaled / factor + smooth * scaled
    medium = (wl >= hi_wl) & (wl <= lo_wl)
    return torch.where(medium, smoothed, scaled)
  if kind == "linear":
    return inv / float(scaling.get("factor", 1.0))
  if kind == "yarn":  # HF _compute_yarn_parameters (DeepSeek-V2/V3)
    dim, base = head_dim, theta
    factor = float(scaling["factor"])
    orig = float(scaling["original_max_position_embeddings"])
    beta_fast, beta_slow = float(scaling.get("beta_fast") or 32), float(scaling.get("beta_slow") or 1)

    def corr(rot):
      return (dim * math.log(orig / (rot * 2 * math.pi))) / (2 * math.log(base))
    lo, hi = corr(beta_fast), corr(beta_slow)
    if scaling.get("truncate", True):
      lo, hi = math.floor(lo), math.ceil(hi)
    lo, hi = max(lo, 0), min(hi, dim - 1)
    if lo == hi:
      hi += 0.001
    ramp = ((torch.arange(dim // 2, dtype=torch.float64) - lo) / (hi - lo)).clamp(0, 1)
    extrap = 1.0 - ramp
    pos_freqs = base ** (torch.arange(0, dim, 2, dtype=torch.float64) / dim)
    return (1.0 / (factor * pos_freqs)) * (1 - extrap) + (1.0 / pos_freqs) * extrap
  return inv


def yarn_attention_factor(scaling: dict | None) -> float:
  """The factor HF YaRN multiplies cos / sin by (1 for DeepSeek, whose mscale == mscale_all_dim)."""
  if not scaling or scaling.get("rope_type") != "yarn":
    return 1.0
  if scaling.get("attention_factor") is not None:
    return float(scaling["attention_factor"])
  f = float(scaling["factor"])

  def ms(scale, m=1.0):
    return 1.0 if scale <= 1 else 0.1 * m * math.log(scale) + 1.0
  m, mad = scaling.get("mscale"), scaling.get("mscale_all_dim")
  if m and mad:
    return ms(f, float(m)) / ms(f, float(mad))
  return ms(f)


def build_cos_sin(head_dim: int, max_pos: int, theta: float = 10000.0, scaling: dict | None = None,
                  device: torch.device | str = "cpu", rotary_dim: Optional[int] = None) -> torch.Tensor:
  """[max_pos, head_dim] fp32 table, row p = [cos(p*f_0..f_{h-1}) | sin(p*f_0..f_{h-1})], h = head_dim / 2.
  With rotary_dim R < head_dim only the first R/2 frequency slots rotate (the rest are cos 1 / sin 0)."""
  R = rotary_dim or head_dim
  pos = torch.arange(max_pos, dtype=torch.float64)
  kind = (scaling or {}).get("rope_type", (scaling or {}).get("type", "default"))
  if kind == "longrope":
    # HF _compute_longrope_parameters: short_factor while the sequence fits the pretraining window,
    # long_factor beyond it (which one a step uses: rope_shift); cos / sin carry the attention factor
    orig = int(scaling["original_max_position_embeddings"])
    factor = scaling.get("factor") or float(scaling.get("max_position_embeddings", orig)) / orig
    attn = scaling.get("attention_factor")
    if attn is None:
      attn = 1.0 if factor <= 1.0 else math.sqrt(1 + math.log(factor) / math.log(orig))
    base = theta ** (torch.arange(0, R, 2, dtype=torch.float64) / R)
    inv_s = 1.0 / (torch.tensor(scaling["short_factor"], dtype=torch.float64) * base)
    inv_l = 1.0 / (torch.tensor(scaling["long_factor"], dtype=torch.float64) * base)
    # rows [0, max_pos): short factors; rows [max_pos, 2 max_pos): long factors (rope_shift picks)
    ang = torch.cat([torch.outer(pos, inv_s), torch.outer(pos, inv_l)], 0)
    cos, sin = ang.cos() * attn, ang.sin() * attn
  else:
    ang = torch.outer(pos, inv_frequencies(R, theta, scaling))
    af = yarn_attention_factor(scaling)
    cos, sin = ang.cos() * af, ang.sin() * af
  if R < head_dim:
    pad = head_dim // 2 - R // 2
    cos = torch.cat([cos, torch.ones(cos.shape[0], pad, dtype=cos.dtype)], 1)
    sin = torch.cat([sin, torch.zeros(sin.shape[0], pad, dtype=sin.dtype)], 1)
  return torch.cat([cos, sin], dim=1).to(torch.float32).to(device).contiguous()


def rope_table(c, max_pos: int, device: torch.device | str = "cpu") -> torch.Tensor:
  """The table for a ModelConfig (rotary dims, scaling and theta from the config; MLA models rotate
  their qk_rope_head_dim slice).  LongRoPE tables hold 2 max_pos rows: the short-factor rows, then the
  long-factor rows (see rope_shift)."""
  return build_cos_sin(c.rope_dim, max_pos, c.rope_theta, c.rope_scaling, device, rotary_dim=c.rotary_dim)


def interleave_perm(d: int) -> torch.Tensor:
  """DeepSeek rotates interleaved pairs (2j, 2j+1): kernel dim p <- HF dim perm[p] = evens, then odds,
  so the pairs become the kernels' rotate-half pairs (j, j + d/2)."""
  return torch.cat([torch.arange(0, d, 2), torch.arange(1, d, 2)])


def longrope_window(c) -> Optional[int]:
  s = c.rope_scaling or {}
  if s.get("rope_type") == "longrope":
    return int(s["original_max_position_embeddings"])
  return None


def rope_shift(window: Optional[int], max_pos: int, total_len: int) -> int:
  """Row offset into a LongRoPE table for a step that leaves a sequence `total_len` tokens long.
  HF Phi-3 rotates a whole forward with the long factors once its sequence exceeds the pretraining
  window (Phi3ForCausalLM.prepare_inputs_for_generation even recomputes the cache at the switch); here a
  step's new tokens follow the same rule, so a prompt longer than the window prefills entirely with the
  long factors (= HF).  Deviation: the keys cached before a sequence crosses the window mid-generation
  keep their short-factor rotation (HF re-runs the prefix at that single token)."""
  return max_pos if window is not None and total_len > window else 0


def rope_perm(head_dim: int, rotary_dim: int) -> Optional[torch.Tensor]:
  """Kernel-order dim p of a head <- HF dim perm[p] (None when every dim rotates)."""
  Dh, R = head_dim, rotary_dim
  if R >= Dh:
    return None
  h, r = Dh // 2, R // 2
  perm = []
  for p in range(Dh):
    q = p if p < h else p - h
    if q < r:
      perm.append(q + (0 if p < h else r))
    else:
      perm.append(R + (q - r) + (0 if p < h else h - r))
  return torch.tensor(perm, dtype=torch.long)


def permute_qk_rows(qkv: torch.Tensor, H: int, Hkv: int, Dh: int, R: int, inverse: bool = False) -> torch.Tensor:
  """Apply rope_perm to the q and k rows of a fused [(H + 2 Hkv) Dh, ...] projection weight / bias."""
  perm = rope_perm(Dh, R)
  if perm is None:
    return qkv
  if inverse:
    perm = torch.argsort(perm)
  nqk = (H + Hkv) * Dh
  idx = (torch.arange(H + Hkv)[:, None] * Dh + perm[None, :]).reshape(-1).to(qkv.device)
  out = qkv.clone()
  out[:nqk] = qkv[:nqk].index_select(0, idx)
  return out

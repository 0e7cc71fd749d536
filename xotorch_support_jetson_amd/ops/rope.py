"""Rotary-embedding tables (host-built once per model, consumed by the RoPE kernels).

Supports plain RoPE (Qwen2/Mistral/Llama-3 without scaling), Llama-3.1/3.2 "llama3" frequency
scaling and linear scaling.  The reference picks torchtune RoPE classes by model-id substring and
reads the wrong config key ("rope_factor") for Llama scaling (xotorch/inference/torch/models/
general_mha.py:33-63, llm_utils.py:68-69); here the HF `rope_scaling` dict is honoured as written and
a missing dict means no scaling (so Llama-3-8B/70B build; the reference KeyErrors on them).
"""
from __future__ import annotations

import math

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
  return inv


def build_cos_sin(head_dim: int, max_pos: int, theta: float = 10000.0, scaling: dict | None = None,
                  device: torch.device | str = "cpu") -> torch.Tensor:
  """[max_pos, head_dim] fp32 table, row p = [cos(p*f_0..f_{h-1}) | sin(p*f_0..f_{h-1})]."""
  inv = inv_frequencies(head_dim, theta, scaling)
  pos = torch.arange(max_pos, dtype=torch.float64)
  ang = torch.outer(pos, inv)
  return torch.cat([ang.cos(), ang.sin()], dim=1).to(torch.float32).to(device).contiguous()

"""Per-shard weights in the fused device layout, built from HF safetensors or random init.

Device layout per decoder layer (all bf16, nn.Linear [out, in] rows):
  qkv_w  [(H + 2 Hkv) Dh, D]   = cat(q_proj, k_proj, v_proj)     (+ qkv_b for Qwen2)
  o_w    [D, H Dh]
  gu_w   [2F, D]               gate/up interleaved in 16-row tiles (one MFMA n-tile each), so the
                               GEMM epilogue computes silu(gate)*up without another pass
  down_w [D, F]
  ln1, ln2 [D]
MoE (Mixtral): router [E, D], gu_w [E, 2F, D], down_w [E, D, F].
Only this shard's layers are materialised (the reference allocates every shard's full embedding and
LM head, general_mha.py:124-128; here the embedding lives on the first shard and the head on the last).
HF names are kept for loading and checkpointing so any shard checkpoint can be re-partitioned.
Reference parity: load_model_weights_torchtune (llm_utils.py:136-284) — without the q/k permute,
because the RoPE kernel uses the HF rotate-half convention directly.
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass, field
from pathlib import Path
from typing import Dict, Iterable, Optional

import torch

from ..inference.shard import Shard
from .config import ModelConfig

TILE = 16


def interleave_gate_up(gate: torch.Tensor, up: torch.Tensor) -> torch.Tensor:
  """[F, D] x2 -> [2F, D] with rows [g0..g15, u0..u15, g16..g31, u16..u31, ...]."""
  Fd, D = gate.shape
  assert Fd % TILE == 0, "intermediate size must be a multiple of 16"
  return torch.stack([gate.view(Fd // TILE, TILE, D), up.view(Fd // TILE, TILE, D)], dim=1).reshape(2 * Fd, D)


def split_gate_up(gu: torch.Tensor):
  n2, D = gu.shape[-2], gu.shape[-1]
  v = gu.reshape(*gu.shape[:-2], n2 // (2 * TILE), 2, TILE, D)
  return v[..., 0, :, :].reshape(*gu.shape[:-2], n2 // 2, D), v[..., 1, :, :].reshape(*gu.shape[:-2], n2 // 2, D)


@dataclass
class LayerWeights:
  qkv_w: torch.Tensor
  o_w: torch.Tensor
  gu_w: torch.Tensor
  down_w: torch.Tensor
  ln1: torch.Tensor
  ln2: torch.Tensor
  qkv_b: Optional[torch.Tensor] = None
  router: Optional[torch.Tensor] = None  # MoE
  # DeepSeek MLA: qkv_w is the fused A projection [q_a (or q) | kv latent | shared rope key]
  q_ln: Optional[torch.Tensor] = None  # [q_lora_rank]
  kv_ln: Optional[torch.Tensor] = None  # [kv_lora_rank]
  qb_w: Optional[torch.Tensor] = None  # [H (dn + dr), q_lora_rank], rows [all heads' nope | all heads' rope]
  wuk: Optional[torch.Tensor] = None  # [H, dn, kv_lora_rank]  (kv_b_proj's key rows, absorbed into q)
  wuv: Optional[torch.Tensor] = None  # [H, dv, kv_lora_rank]  (kv_b_proj's value rows)
  # DeepSeekMoE
  router_bias: Optional[torch.Tensor] = None  # [E] fp32 selection bias (V3 e_score_correction_bias)
  sh_gu_w: Optional[torch.Tensor] = None  # shared experts, gate/up interleaved [2 Fs, D]
  sh_down_w: Optional[torch.Tensor] = None  # [D, Fs]

  def tensors(self) -> Dict[str, torch.Tensor]:
    return {k: v for k, v in self.__dict__.items() if isinstance(v, torch.Tensor)}


@dataclass
class ShardWeights:
  config: ModelConfig
  shard: Shard
  layers: Dict[int, LayerWeights] = field(default_factory=dict)
  embed: Optional[torch.Tensor] = None  # first shard (and last, when tied)
  norm: Optional[torch.Tensor] = None  # last shard
  lm_head: Optional[torch.Tensor] = None  # last shard (aliases embed when tied)
  vision: Optional[Dict[str, torch.Tensor]] = None  # LLaVA tower + projector (first shard), HF names

  def nbytes(self) -> int:
    seen, total = set(), 0
    for t in self.all_tensors():
      if t.data_ptr() not in seen:
        seen.add(t.data_ptr())
        total += t.numel() * t.element_size()
    return total

  def all_tensors(self) -> Iterable[torch.Tensor]:
    for lw in self.layers.values():
      yield from lw.tensors().values()
    for t in (self.embed, self.norm, self.lm_head):
      if t is not None:
        yield t
    if self.vision:
      yield from self.vision.values()

  # ---------------------------------------------------------------- HF naming (checkpoints)
  def to_hf_state_dict(self) -> Dict[str, torch.Tensor]:
    c = self.config
    H, Hkv, Dh = c.num_heads, c.num_kv_heads, c.head_dim
    sd: Dict[str, torch.Tensor] = {}
    from ..ops.rope import permute_qk_rows
    fused = c.model_type == "phi3"  # Phi-3 checkpoints keep qkv_proj / gate_up_proj fused
    for i, lw in self.layers.items():
      p = f"model.layers.{i}."
      if c.is_mla:
        _mla_to_hf(c, lw, p, sd)
        continue
      qkv_w = permute_qk_rows(_rowmajor(lw.qkv_w), H, Hkv, Dh, c.rotary_dim, inverse=True)
      if fused:
        sd[p + "self_attn.qkv_proj.weight"] = qkv_w
      else:
        q, k, v = qkv_w.split([H * Dh, Hkv * Dh, Hkv * Dh], 0)
        sd[p + "self_attn.q_proj.weight"], sd[p + "self_attn.k_proj.weight"], sd[p + "self_attn.v_proj.weight"] = q, k, v
      if lw.qkv_b is not None:
        qkv_b = permute_qk_rows(lw.qkv_b, H, Hkv, Dh, c.rotary_dim, inverse=True)
        qb, kb, vb = qkv_b.split([H * Dh, Hkv * Dh, Hkv * Dh], 0)
        sd[p + "self_attn.q_proj.bias"], sd[p + "self_attn.k_proj.bias"], sd[p + "self_attn.v_proj.bias"] = qb, kb, vb
      sd[p + "self_attn.o_proj.weight"] = _rowmajor(lw.o_w)
      sd[p + "input_layernorm.weight"] = lw.ln1
      sd[p + "post_attention_layernorm.weight"] = lw.ln2
      gu, down = _rowmajor(lw.gu_w), _rowmajor(lw.down_w)
      if c.is_moe:
        sd[p + "block_sparse_moe.gate.weight"] = lw.router
        g, u = split_gate_up(gu)
        for e in range(c.num_experts):
          sd[p + f"block_sparse_moe.experts.{e}.w1.weight"] = g[e]
          sd[p + f"block_sparse_moe.experts.{e}.w3.weight"] = u[e]
          sd[p + f"block_sparse_moe.experts.{e}.w2.weight"] = down[e]
      else:
        g, u = split_gate_up(gu)
        if fused:
          sd[p + "mlp.gate_up_proj.weight"] = torch.cat([g, u], 0)
        else:
          sd[p + "mlp.gate_proj.weight"], sd[p + "mlp.up_proj.weight"] = g, u
        sd[p + "mlp.down_proj.weight"] = down
    if self.embed is not None:
      sd["model.embed_tokens.weight"] = self.embed
    if self.norm is not None:
      sd["model.norm.weight"] = self.norm
    if self.lm_head is not None and not c.tie_word_embeddings:
      sd["lm_head.weight"] = _rowmajor(self.lm_head)
    elif self.lm_head is not None and self.embed is None:
      sd["model.embed_tokens.weight"] = _rowmajor(self.lm_head)  # tied head on a shard without the embedding
    if self.vision:
      sd.update(self.vision)
    return {k: v.contiguous() for k, v in sd.items()}


def _mla_q_order(c: ModelConfig) -> torch.Tensor:
  """Device row r of the q projection <- HF row: all heads' nope dims, then all heads' rope dims with the
  interleaved pairs de-interleaved (ops.rope.interleave_perm)."""
  from ..ops.rope import interleave_perm
  H, dn, dr = c.num_heads, c.qk_nope_head_dim, c.qk_rope_head_dim
  hd = dn + dr
  nope = (torch.arange(H)[:, None] * hd + torch.arange(dn)[None, :]).reshape(-1)
  rope = (torch.arange(H)[:, None] * hd + dn + interleave_perm(dr)[None, :]).reshape(-1)
  return torch.cat([nope, rope])


def _mla_kv_order(c: ModelConfig) -> torch.Tensor:
  from ..ops.rope import interleave_perm
  L = c.kv_lora_rank
  return torch.cat([torch.arange(L), L + interleave_perm(c.qk_rope_head_dim)])


def _mla_from_hf(c: ModelConfig, get, has, p: str) -> dict:
  """HF DeepSeek attention tensors -> device layout fields of LayerWeights."""
  a = p + "self_attn."
  qo = _mla_q_order(c)
  kv_a = get(a + "kv_a_proj_with_mqa.weight")
  kv_a = kv_a.index_select(0, _mla_kv_order(c).to(kv_a.device))
  out = {}
  if c.q_lora_rank:
    q_a = get(a + "q_a_proj.weight")
    out["q_ln"] = get(a + "q_a_layernorm.weight")
    qb = get(a + "q_b_proj.weight")
    out["qb_w"] = qb.index_select(0, qo.to(qb.device)).contiguous()
  else:
    q = get(a + "q_proj.weight")
    q_a = q.index_select(0, qo.to(q.device))
  out["qkv_w"] = torch.cat([q_a, kv_a], 0).contiguous()
  out["kv_ln"] = get(a + "kv_a_layernorm.weight")
  kvb = get(a + "kv_b_proj.weight").view(c.num_heads, c.qk_nope_head_dim + c.v_head_dim, c.kv_lora_rank)
  out["wuk"] = kvb[:, :c.qk_nope_head_dim].contiguous()
  out["wuv"] = kvb[:, c.qk_nope_head_dim:].contiguous()
  out["o_w"] = get(a + "o_proj.weight")
  return out


def _mla_to_hf(c: ModelConfig, lw: "LayerWeights", p: str, sd: Dict[str, torch.Tensor]) -> None:
  a = p + "self_attn."
  qo = torch.argsort(_mla_q_order(c))
  ko = torch.argsort(_mla_kv_order(c))
  A = _rowmajor(lw.qkv_w)
  nq = c.q_lora_rank or c.num_heads * (c.qk_nope_head_dim + c.qk_rope_head_dim)
  q_a, kv_a = A[:nq], A[nq:]
  sd[a + "kv_a_proj_with_mqa.weight"] = kv_a.index_select(0, ko.to(kv_a.device))
  if c.q_lora_rank:
    sd[a + "q_a_proj.weight"] = q_a
    sd[a + "q_a_layernorm.weight"] = lw.q_ln
    qb = _rowmajor(lw.qb_w)
    sd[a + "q_b_proj.weight"] = qb.index_select(0, qo.to(qb.device))
  else:
    sd[a + "q_proj.weight"] = q_a.index_select(0, qo.to(q_a.device))
  sd[a + "kv_a_layernorm.weight"] = lw.kv_ln
  sd[a + "kv_b_proj.weight"] = torch.cat([_rowmajor(lw.wuk), _rowmajor(lw.wuv)], 1).reshape(-1, c.kv_lora_rank)
  sd[a + "o_proj.weight"] = _rowmajor(lw.o_w)
  sd[p + "input_layernorm.weight"] = lw.ln1
  sd[p + "post_attention_layernorm.weight"] = lw.ln2
  gu, down = _rowmajor(lw.gu_w), _rowmajor(lw.down_w)
  g, u = split_gate_up(gu)
  if lw.router is not None:
    m = p + "mlp."
    sd[m + "gate.weight"] = lw.router
    if lw.router_bias is not None:
      sd[m + "gate.e_score_correction_bias"] = lw.router_bias
    for e in range(c.num_experts):
      sd[m + f"experts.{e}.gate_proj.weight"], sd[m + f"experts.{e}.up_proj.weight"] = g[e], u[e]
      sd[m + f"experts.{e}.down_proj.weight"] = down[e]
    if lw.sh_gu_w is not None:
      sg, su = split_gate_up(_rowmajor(lw.sh_gu_w))
      sd[m + "shared_experts.gate_proj.weight"], sd[m + "shared_experts.up_proj.weight"] = sg, su
      sd[m + "shared_experts.down_proj.weight"] = _rowmajor(lw.sh_down_w)
  else:
    sd[p + "mlp.gate_proj.weight"], sd[p + "mlp.up_proj.weight"] = g, u
    sd[p + "mlp.down_proj.weight"] = down


def _rowmajor(t: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
  """Row-major view of a possibly pre-shuffled device weight (2-D, or 3-D expert stacks), without the zero
  padding a tiled layout may carry (`xot_logical`: see pad_ffn_for_tiles)."""
  logical = getattr(t, "xot_logical", None)
  if logical is not None:
    full = _rowmajor_full(t)
    return full[:logical[0], :logical[1]].contiguous()
  return _rowmajor_full(t)


def _rowmajor_full(t: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
  if t is not None and getattr(t, "xot_layout", "rowmajor") == "stream8":
    from ..ops.weights_layout import dequant_stream8
    return dequant_stream8(t, t.xot_scale)
  if t is not None and getattr(t, "xot_layout", "rowmajor") == "stream_t":  # per-head shuffled W^T (MLA W_UK)
    from ..ops.weights_layout import unshuffle_from_stream
    return torch.stack([unshuffle_from_stream(t[h]).t() for h in range(t.shape[0])])
  if t is None or getattr(t, "xot_layout", "rowmajor") != "stream":
    return t
  from ..ops.weights_layout import unshuffle_from_stream
  if t.dim() == 3:
    return torch.stack([unshuffle_from_stream(t[e]) for e in range(t.shape[0])])
  return unshuffle_from_stream(t)


def expert(t: torch.Tensor, e: int) -> torch.Tensor:
  """Expert e's [rows, K] weight, keeping the storage-layout tag of the stack."""
  v = t[e]
  if hasattr(t, "xot_layout"):
    v.xot_layout = t.xot_layout
  return v


def _pad_to(t: torch.Tensor, shape) -> torch.Tensor:
  """Zero-pad the trailing rows / columns of a 2-D tensor up to `shape`."""
  return torch.nn.functional.pad(t, (0, shape[1] - t.shape[1], 0, shape[0] - t.shape[0]))


def pad_ffn_for_tiles(lw: "LayerWeights") -> None:
  """A dense SwiGLU whose intermediate size F is not a multiple of 128 (DeepSeek-V2-Lite's first layer:
  10944) cannot take the down projection (K = F) on the 128-deep pre-shuffled tiles.  Pad F to F' = 128k
  with zero features instead: gate/up gain zero rows (interleaved groups past F, so silu(0) * 0 = 0 columns
  in the activation) and down gains zero columns -- the same products, every GEMM on the tiled kernels.
  `xot_logical` records the unpadded shape for _rowmajor / assign_weight (training, export)."""
  gu, down = lw.gu_w, lw.down_w
  if gu is None or down is None or gu.dim() != 2 or lw.router is not None or not gu.is_cuda:
    return
  if getattr(gu, "xot_layout", "rowmajor") != "rowmajor" or getattr(down, "xot_layout", "rowmajor") != "rowmajor":
    return
  F = down.shape[1]
  if F % 128 == 0 or F % TILE or gu.shape[0] != 2 * F:
    return
  Fp = -(-F // 128) * 128
  lw.gu_w = _pad_to(gu, (2 * Fp, gu.shape[1]))  # pad rows after the last interleaved (gate, up) group pair
  lw.down_w = _pad_to(down, (down.shape[0], Fp))
  lw.gu_w.xot_logical, lw.down_w.xot_logical = tuple(gu.shape), tuple(down.shape)


def prepare_for_decode(sw: "ShardWeights", keep_rowmajor: Iterable[str] = (), fp8: bool = False) -> "ShardWeights":
  """Convert the projection weights of a GPU shard to the pre-shuffled stream layout (in place).
  The embedding stays row-major (it is gathered); a tied LM head gets its own shuffled copy.
  `keep_rowmajor` names projections ("qkv", "o", "gu", "down") left row-major: at decode batches of
  ~256 rows hipBLASLt beats the stream GEMM on the wide qkv / gate-up shapes, while the stream GEMM
  keeps winning on o / down (tools/bench_gemm_m.py, profiles/bench_gemm_m_*.json)."""
  keep = set(keep_rowmajor)
  from ..ops.weights_layout import can_shuffle, shuffle_for_stream
  from ..ops.linear import to_stream8_layout
  if sw.embed is not None and not sw.embed.is_cuda:
    return sw
  if sw.lm_head is None and not sw.layers:
    return sw

  def conv(t):
    if t is None or not t.is_cuda or getattr(t, "xot_layout", "rowmajor") == "stream":
      return t
    if t.dim() == 3:
      if not all(can_shuffle(t[e]) for e in range(t.shape[0])):
        return t
      out = torch.empty_like(t)
      for e in range(t.shape[0]):
        out[e] = shuffle_for_stream(t[e])
    else:
      if not can_shuffle(t):
        return t
      out = shuffle_for_stream(t)
    out.xot_layout = "stream"
    return out

  def conv8(t):  # fp8=True: the dense projections become weight-only FP8 (experts, latent and LM head stay bf16)
    if t is None or not t.is_cuda or t.dim() != 2 or getattr(t, "xot_layout", "rowmajor") != "rowmajor":
      return conv(t)
    return to_stream8_layout(t) if can_shuffle(t) else t

  def conv_bat(t, transpose: bool):
    """MLA absorbed projections for gemm_batched (N % 128 == 0): W_UV [H, dv, L] per head shuffled ("stream");
    W_UK [H, dn, L] -> per head shuffle(W_UK[h]^T) [H, L, dn] ("stream_t"), so q_lat = q_nope . W_UK is Y = X W^T."""
    if t is None or not t.is_cuda or getattr(t, "xot_layout", "rowmajor") != "rowmajor":
      return t
    ws = [t[h].t() if transpose else t[h] for h in range(t.shape[0])]
    if not all(can_shuffle(w) and w.shape[0] % 128 == 0 for w in ws):
      return t
    out = torch.stack([shuffle_for_stream(w.contiguous()) for w in ws])
    out.xot_layout = "stream_t" if transpose else "stream"
    return out

  proj = conv8 if fp8 else conv

  def keep_logical(new, old):  # a converted weight keeps the padded tensor's logical shape
    if new is not old and getattr(old, "xot_logical", None) is not None:
      new.xot_logical = old.xot_logical
    return new

  for lw in sw.layers.values():
    if ("gu" not in keep and "down" not in keep) or fp8:
      pad_ffn_for_tiles(lw)
    g0, d0 = lw.gu_w, lw.down_w
    lw.qb_w, lw.sh_gu_w, lw.sh_down_w = conv(lw.qb_w), conv(lw.sh_gu_w), conv(lw.sh_down_w)
    lw.wuk, lw.wuv = conv_bat(lw.wuk, True), conv_bat(lw.wuv, False)  # the absorbed MLA projections run on gemm_batched
    if "qkv" not in keep or fp8:
      lw.qkv_w = proj(lw.qkv_w)
    if "o" not in keep or fp8:
      lw.o_w = proj(lw.o_w)
    if "gu" not in keep or fp8:
      lw.gu_w = proj(lw.gu_w)
    if "down" not in keep or fp8:
      lw.down_w = proj(lw.down_w)
    lw.gu_w, lw.down_w = keep_logical(lw.gu_w, g0), keep_logical(lw.down_w, d0)
  if sw.lm_head is not None:
    sw.lm_head = conv(sw.lm_head)  # a tied head becomes a separate shuffled copy; embed stays row-major
  return sw


@torch.no_grad()
def assign_weight(dst: Optional[torch.Tensor], src: torch.Tensor) -> None:
  """Write a row-major `src` into `dst` IN PLACE, honouring dst's storage layout (pre-shuffled or
  not).  In-place matters: captured HIP graphs hold the addresses of the inference weights."""
  if dst is None:
    return
  if getattr(dst, "xot_layout", "rowmajor") == "stream8":  # re-quantize (new row scales, same storage)
    from ..ops.weights_layout import quantize_fp8_rows, shuffle_for_stream8
    if getattr(dst, "xot_logical", None) is not None:
      src = _pad_to(src, dst.shape)
    q, sc = quantize_fp8_rows(src.to(dst.device))
    dst.copy_(shuffle_for_stream8(q))
    dst.xot_scale.copy_(sc)
    return
  src = src.to(device=dst.device, dtype=dst.dtype)
  if getattr(dst, "xot_logical", None) is not None and tuple(src.shape) != tuple(dst.shape):
    src = _pad_to(src, dst.shape)
  if getattr(dst, "xot_layout", "rowmajor") == "stream_t":
    from ..ops.weights_layout import shuffle_for_stream
    for h in range(dst.shape[0]):
      dst[h].copy_(shuffle_for_stream(src[h].t().contiguous()))
  elif getattr(dst, "xot_layout", "rowmajor") == "stream":
    from ..ops.weights_layout import shuffle_for_stream
    if dst.dim() == 3:
      for e in range(dst.shape[0]):
        dst[e].copy_(shuffle_for_stream(src[e]))
    else:
      dst.copy_(shuffle_for_stream(src))
  else:
    dst.copy_(src)


@torch.no_grad()
def copy_weights_into(dst: "ShardWeights", src: "ShardWeights") -> None:
  """Copy every tensor of the row-major `src` shard into the live inference shard `dst` in place."""
  for i, lw in dst.layers.items():
    s = src.layers[i]
    for name in ("qkv_w", "o_w", "gu_w", "down_w", "ln1", "ln2", "qkv_b", "router", "q_ln", "kv_ln", "qb_w", "wuk",
                 "wuv", "router_bias", "sh_gu_w", "sh_down_w"):
      if getattr(lw, name) is not None and getattr(s, name) is not None:
        assign_weight(getattr(lw, name), getattr(s, name))
  if dst.embed is not None and src.embed is not None:
    assign_weight(dst.embed, src.embed)
  if dst.norm is not None and src.norm is not None:
    assign_weight(dst.norm, src.norm)
  if dst.lm_head is not None and dst.lm_head is not dst.embed:
    head = src.lm_head if src.lm_head is not None else src.embed
    if head is not None:
      assign_weight(dst.lm_head, head)


def _needs_embed(c: ModelConfig, s: Shard) -> bool:
  return s.is_first_layer() or (s.is_last_layer() and c.tie_word_embeddings)


# -------------------------------------------------------------------- random init
def _normal(shape, g: torch.Generator, std: float, dev: torch.device, dtype) -> torch.Tensor:
  """N(0, std) of `shape` from generator g; every random weight (and random_head_rows) draws through here, so a
  shard's rows are the same whichever function made them.  (Drawing CPU bf16 weights in fp32 and rounding is ~3x
  faster, but it changes every value, and the exact-equality training tests are pinned to these.)"""
  return torch.empty(shape, device=dev, dtype=dtype).normal_(0.0, std, generator=g)


def random_weights(c: ModelConfig, shard: Shard, device: torch.device | str = "cpu", dtype=torch.bfloat16,
                   seed: int = 0, std: float = 0.02) -> ShardWeights:
  """Deterministic per-layer random weights: layer i is identical whichever shard holds it, so a
  pipeline split reproduces the unsplit model exactly (the split-vs-full equivalence tests)."""
  dev = torch.device(device)
  D, Fd, E = c.hidden_size, c.intermediate_size, c.num_experts

  def gen(tag: int):
    g = torch.Generator(device=dev)
    g.manual_seed(seed * 1_000_003 + tag)
    return g

  def normal(shape, g, s=std):
    return _normal(shape, g, s, dev, dtype)

  def norm_w(g):
    return (1.0 + torch.empty(D, device=dev, dtype=torch.float32).normal_(0.0, 0.05, generator=g)).to(dtype)

  def vec(n, g):
    return (1.0 + torch.empty(n, device=dev, dtype=torch.float32).normal_(0.0, 0.05, generator=g)).to(dtype)

  sw = ShardWeights(c, shard)
  for i in shard.layers():
    g = gen(1000 + i)
    out_std = std / (2 * c.num_layers) ** 0.5  # GPT-2 style residual-branch scaling keeps deep stacks stable
    moe = c.moe_layer(i)
    Fl = c.expert_dim if moe else Fd
    El = E if moe else 0
    lw = LayerWeights(
      qkv_w=normal((c.qkv_size, D), g),
      o_w=normal((D, c.num_heads * (c.v_head_dim if c.is_mla else c.head_dim)), g, out_std),
      gu_w=normal((El, 2 * Fl, D) if El else (2 * Fl, D), g),
      down_w=normal((El, D, Fl) if El else (D, Fl), g, out_std),
      ln1=norm_w(g),
      ln2=norm_w(g),
      qkv_b=normal((c.qkv_size,), g) if c.attention_bias and not c.is_mla else None,
      router=normal((El, D), g, 0.1) if El else None,
    )
    if c.is_mla:
      H, L = c.num_heads, c.kv_lora_rank
      if c.q_lora_rank:
        lw.q_ln = vec(c.q_lora_rank, g)
        lw.qb_w = normal((H * (c.qk_nope_head_dim + c.qk_rope_head_dim), c.q_lora_rank), g)
      lw.kv_ln = vec(L, g)
      lw.wuk = normal((H, c.qk_nope_head_dim, L), g)
      lw.wuv = normal((H, c.v_head_dim, L), g)
    if moe and c.scoring_func == "sigmoid":
      lw.router_bias = torch.empty(El, device=dev, dtype=torch.float32).normal_(0.0, 0.01, generator=g)
    if moe and c.n_shared_experts:
      Fs = c.n_shared_experts * c.expert_dim
      lw.sh_gu_w = normal((2 * Fs, D), g)
      lw.sh_down_w = normal((D, Fs), g, out_std)
    sw.layers[i] = lw
  if _needs_embed(c, shard):
    sw.embed = normal((c.vocab_size, D), gen(1))
  if shard.is_last_layer():
    sw.norm = norm_w(gen(2))
    sw.lm_head = sw.embed if c.tie_word_embeddings else normal((c.vocab_size, D), gen(3))
  if c.vision and shard.is_first_layer():
    from .vision import random_vision
    sw.vision = random_vision(c, dev, dtype, seed=seed)
  return sw


def random_head_rows(c: ModelConfig, rows_from: int, device: torch.device | str = "cpu", dtype=torch.bfloat16,
                     seed: int = 0, std: float = 0.02) -> torch.Tensor:
  """Rows [rows_from, V) of the LM head random_weights gives the last shard (same generator stream, so
  a stage holding only these rows computes exactly the full head's logits for them)."""
  dev = torch.device(device)
  g = torch.Generator(device=dev)
  g.manual_seed(seed * 1_000_003 + (1 if c.tie_word_embeddings else 3))
  full = _normal((c.vocab_size, c.hidden_size), g, std, dev, dtype)
  return full[rows_from:].clone()


# -------------------------------------------------------------------- HF safetensors
def _weight_map(model_dir: Path) -> Dict[str, str]:
  idx = model_dir / "model.safetensors.index.json"
  if idx.exists():
    return json.loads(idx.read_text())["weight_map"]
  files = sorted(model_dir.glob("*.safetensors"))
  if not files:
    raise FileNotFoundError(f"no safetensors in {model_dir}")
  from safetensors import safe_open
  wm = {}
  for f in files:
    with safe_open(str(f), framework="pt") as sf:
      for k in sf.keys():
        wm[k] = f.name
  return wm


_PREFIXES = (("language_model.model.", "model."), ("language_model.lm_head.", "lm_head."),
             ("model.language_model.", "model."), ("model.vision_tower.", "vision_tower."),
             ("model.multi_modal_projector.", "multi_modal_projector."), ("vision_tower.vision_model.", "vision_tower."))


def canonical_name(k: str) -> str:
  """One name per tensor across checkpoint flavours: LLaVA's `language_model.model.*` (hub) /
  `model.language_model.*` (transformers 5) read as the plain LM's `model.*`, the hub's
  `vision_tower.vision_model.*` as `vision_tower.*`."""
  changed = True
  while changed:
    changed = False
    for a, b in _PREFIXES:
      if k.startswith(a):
        k, changed = b + k[len(a):], True
  return k


def needed_files(model_dir: Path, c: ModelConfig, shard: Shard) -> set:
  """Safetensors files that hold this shard's tensors (for the downloader's allow patterns too)."""
  wm = {canonical_name(k): v for k, v in _weight_map(model_dir).items()}
  want = set()
  for name, fname in wm.items():
    if (name.startswith("vision_tower.") or name.startswith("multi_modal_projector.")) and shard.is_first_layer():
      want.add(fname)
    elif name.startswith("model.layers."):
      if int(name.split(".")[2]) in shard.layers():
        want.add(fname)
    elif name.startswith("model.embed_tokens") and _needs_embed(c, shard):
      want.add(fname)
    elif (name.startswith("model.norm") or name.startswith("lm_head")) and shard.is_last_layer():
      want.add(fname)
  return want


def load_hf_weights(model_dir: str | Path, c: ModelConfig, shard: Shard, device="cpu", dtype=torch.bfloat16) -> ShardWeights:
  """Read only this shard's tensors (mmap'd safetensors, one tensor at a time) into the fused layout."""
  from safetensors import safe_open
  model_dir = Path(model_dir)
  raw = _weight_map(model_dir)
  wm = {canonical_name(k): (k, f) for k, f in raw.items()}
  handles = {}

  def get(name: str, dt: Optional[torch.dtype] = None) -> torch.Tensor:
    key, fname = wm[name]
    if fname not in handles:
      handles[fname] = safe_open(str(model_dir / fname), framework="pt")
    return handles[fname].get_tensor(key).to(device=device, dtype=dt or dtype)

  def has(name: str) -> bool:
    return name in wm

  from ..ops.rope import permute_qk_rows
  H, Hkv, Dh, R = c.num_heads, c.num_kv_heads, c.head_dim, c.rotary_dim
  sw = ShardWeights(c, shard)
  for i in shard.layers():
    p = f"model.layers.{i}."
    if c.is_mla:
      sw.layers[i] = _load_deepseek_layer(c, i, p, get, has)
      continue
    if has(p + "self_attn.qkv_proj.weight"):  # Phi-3: fused [q; k; v]
      qkv = get(p + "self_attn.qkv_proj.weight")
    else:
      qkv = torch.cat([get(p + f"self_attn.{n}_proj.weight") for n in "qkv"], 0)
    qkv = permute_qk_rows(qkv, H, Hkv, Dh, R)  # partial rotary: HF dim order -> the kernels' pair order
    qkv_b = None
    if has(p + "self_attn.q_proj.bias"):
      qkv_b = permute_qk_rows(torch.cat([get(p + f"self_attn.{n}_proj.bias") for n in "qkv"], 0), H, Hkv, Dh, R)
    if c.is_moe:
      pm = p + "block_sparse_moe."
      gu = torch.stack([interleave_gate_up(get(pm + f"experts.{e}.w1.weight"), get(pm + f"experts.{e}.w3.weight"))
                        for e in range(c.num_experts)])
      down = torch.stack([get(pm + f"experts.{e}.w2.weight") for e in range(c.num_experts)])
      router = get(pm + "gate.weight")
    else:
      if has(p + "mlp.gate_up_proj.weight"):  # Phi-3: fused [gate; up]
        gate, up = get(p + "mlp.gate_up_proj.weight").chunk(2, 0)
      else:
        gate, up = get(p + "mlp.gate_proj.weight"), get(p + "mlp.up_proj.weight")
      gu = interleave_gate_up(gate, up)
      down = get(p + "mlp.down_proj.weight")
      router = None
    sw.layers[i] = LayerWeights(qkv.contiguous(), get(p + "self_attn.o_proj.weight"), gu.contiguous(), down,
                                get(p + "input_layernorm.weight"), get(p + "post_attention_layernorm.weight"), qkv_b,
                                router)
  if _needs_embed(c, shard):
    sw.embed = get("model.embed_tokens.weight")
  if shard.is_last_layer():
    sw.norm = get("model.norm.weight")
    if has("lm_head.weight") and not c.tie_word_embeddings:
      sw.lm_head = get("lm_head.weight")
    else:
      sw.lm_head = sw.embed
  if c.vision and shard.is_first_layer():
    from .vision import vision_names
    sw.vision = {n: get(n) for n in vision_names(c.vision)}
  return sw


def _load_deepseek_layer(c: ModelConfig, i: int, p: str, get, has) -> LayerWeights:
  f = _mla_from_hf(c, get, has, p)
  m = p + "mlp."
  lw = LayerWeights(f["qkv_w"], f["o_w"], None, None, get(p + "input_layernorm.weight"),
                    get(p + "post_attention_layernorm.weight"), None, None, f.get("q_ln"), f["kv_ln"], f.get("qb_w"),
                    f["wuk"], f["wuv"])
  if c.moe_layer(i):
    lw.gu_w = torch.stack([interleave_gate_up(get(m + f"experts.{e}.gate_proj.weight"),
                                              get(m + f"experts.{e}.up_proj.weight")) for e in range(c.num_experts)])
    lw.down_w = torch.stack([get(m + f"experts.{e}.down_proj.weight") for e in range(c.num_experts)])
    lw.router = get(m + "gate.weight")
    if has(m + "gate.e_score_correction_bias"):
      lw.router_bias = get(m + "gate.e_score_correction_bias", torch.float32)
    elif c.scoring_func == "sigmoid":
      lw.router_bias = torch.zeros(c.num_experts, dtype=torch.float32, device=lw.router.device)
    if c.n_shared_experts:
      lw.sh_gu_w = interleave_gate_up(get(m + "shared_experts.gate_proj.weight"),
                                      get(m + "shared_experts.up_proj.weight")).contiguous()
      lw.sh_down_w = get(m + "shared_experts.down_proj.weight")
  else:
    lw.gu_w = interleave_gate_up(get(m + "gate_proj.weight"), get(m + "up_proj.weight")).contiguous()
    lw.down_w = get(m + "down_proj.weight")
  return lw


def from_hf_state_dict(sd: Dict[str, torch.Tensor], c: ModelConfig, shard: Shard, device="cpu",
                       dtype=torch.bfloat16) -> ShardWeights:
  """Inverse of ShardWeights.to_hf_state_dict (used by checkpoint resume)."""
  import tempfile
  from safetensors.torch import save_file
  with tempfile.TemporaryDirectory() as d:
    save_file({k: v.contiguous() for k, v in sd.items()}, os.path.join(d, "model.safetensors"))
    return load_hf_weights(d, c, shard, device, dtype)

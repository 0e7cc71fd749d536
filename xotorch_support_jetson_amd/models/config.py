"""Model configuration: HF `config.json` -> typed ModelConfig, plus built-in presets.

Presets carry the public HF architecture numbers for the BASELINE.json configs so the framework can
build random-init models of the exact shape offline (there is no network on the GPU box).
Reference: load_model_config (xotorch/inference/torch/models/llm_utils.py:30-77); unlike it, the
layer count comes from config.json and is validated against the model card.
"""
from __future__ import annotations

import json
from dataclasses import asdict, dataclass, field, replace
from pathlib import Path
from typing import Optional


@dataclass(frozen=True)
class ModelConfig:
  model_type: str  # llama | qwen2 | mistral | mixtral
  vocab_size: int
  hidden_size: int
  intermediate_size: int
  num_layers: int
  num_heads: int
  num_kv_heads: int
  head_dim: int
  rms_norm_eps: float = 1e-5
  rope_theta: float = 500000.0
  rope_scaling: Optional[dict] = None
  max_position_embeddings: int = 8192
  tie_word_embeddings: bool = False
  attention_bias: bool = False
  num_experts: int = 0  # >0: MoE (Mixtral) MLP
  num_experts_per_tok: int = 0
  bos_token_id: int = 128000
  eos_token_ids: tuple = (128001, 128009)
  partial_rotary_factor: float = 1.0  # Phi-3: RoPE on the first 75 % of each head's dims
  # DeepSeek-V2/V3 multi-head latent attention (kv_lora_rank > 0): per token the cache holds one
  # normalised latent [kv_lora_rank] + one shared rotated key [qk_rope_head_dim]
  q_lora_rank: int = 0  # 0: plain q_proj
  kv_lora_rank: int = 0
  qk_nope_head_dim: int = 0
  qk_rope_head_dim: int = 0
  v_head_dim: int = 0
  # MoE routing (Mixtral: softmax top-k renormalised; DeepSeek: shared experts, dense first layers,
  # group-limited selection, sigmoid scores with a selection bias (V3), scaled weights)
  moe_intermediate_size: int = 0  # 0: intermediate_size
  n_shared_experts: int = 0
  first_k_dense_replace: int = 0
  moe_layer_freq: int = 1
  routed_scaling_factor: float = 1.0
  topk_method: str = "greedy"  # greedy | group_limited_greedy (V2) | noaux_tc (V3)
  n_group: int = 1
  topk_group: int = 1
  norm_topk_prob: bool = True
  scoring_func: str = "softmax"  # softmax | sigmoid
  # LLaVA: CLIP vision tower + projector on the first shard (HF vision_config keys), image token id
  vision: Optional[dict] = None
  image_token_id: int = -1
  vision_feature_layer: int = -2
  vision_select: str = "default"  # default: drop the CLS feature | full
  projector_act: str = "gelu"

  @property
  def qkv_size(self) -> int:
    if self.is_mla:  # fused A projection: [q_a (or the full q) | kv_a latent | shared rope key]
      q = self.q_lora_rank or self.num_heads * (self.qk_nope_head_dim + self.qk_rope_head_dim)
      return q + self.kv_lora_rank + self.qk_rope_head_dim
    return (self.num_heads + 2 * self.num_kv_heads) * self.head_dim

  @property
  def is_mla(self) -> bool:
    return self.kv_lora_rank > 0

  @property
  def mla_dim(self) -> int:
    """Latent cache row: normalised kv latent + rotated shared key."""
    return self.kv_lora_rank + self.qk_rope_head_dim

  @property
  def rope_dim(self) -> int:
    return self.qk_rope_head_dim if self.is_mla else self.head_dim

  @property
  def rotary_dim(self) -> int:
    r = int(self.rope_dim * self.partial_rotary_factor)
    return r - (r % 2)

  @property
  def is_moe(self) -> bool:
    return self.num_experts > 0

  @property
  def expert_dim(self) -> int:
    return self.moe_intermediate_size or self.intermediate_size

  def moe_layer(self, i: int) -> bool:
    """Layer i has a routed-expert MLP (HF DeepseekV3DecoderLayer's rule; every layer for Mixtral)."""
    return self.is_moe and i >= self.first_k_dense_replace and i % max(1, self.moe_layer_freq) == 0

  def attn_scale(self) -> float:
    """Softmax scale: 1/sqrt(q.k dim); DeepSeek YaRN multiplies by mscale(factor, mscale_all_dim)^2."""
    import math
    dq = self.qk_nope_head_dim + self.qk_rope_head_dim if self.is_mla else self.head_dim
    s = dq ** -0.5
    sc = self.rope_scaling or {}
    if sc.get("rope_type") == "yarn" and sc.get("mscale_all_dim"):
      f = float(sc.get("factor", 1.0))
      m = 1.0 if f <= 1 else 0.1 * float(sc["mscale_all_dim"]) * math.log(f) + 1.0
      s *= m * m
    return s

  def params_per_layer(self, i: int = -1) -> int:
    D, F = self.hidden_size, self.intermediate_size
    if self.is_mla:
      H, dn, dr, dv = self.num_heads, self.qk_nope_head_dim, self.qk_rope_head_dim, self.v_head_dim
      attn = D * self.qkv_size + (self.q_lora_rank * H * (dn + dr) if self.q_lora_rank else 0)
      attn += self.kv_lora_rank * H * (dn + dv) + H * dv * D
    else:
      attn = D * self.qkv_size + self.num_heads * self.head_dim * D
    moe = self.moe_layer(i) if i >= 0 else self.is_moe
    if moe:
      Fe = self.expert_dim
      mlp = 3 * D * Fe * (self.num_experts + self.n_shared_experts) + D * self.num_experts
    else:
      mlp = 3 * D * F
    return attn + mlp + 2 * D

  def num_params(self) -> int:
    emb = self.vocab_size * self.hidden_size
    layers = sum(self.params_per_layer(i) for i in range(self.num_layers))
    return layers + emb * (1 if self.tie_word_embeddings else 2) + self.hidden_size

  def to_dict(self) -> dict:
    d = asdict(self)
    d["eos_token_ids"] = list(self.eos_token_ids)
    return d

  def with_layers(self, n: int) -> "ModelConfig":
    return replace(self, num_layers=n)


def _rope_fields(cfg: dict) -> tuple:
  """(theta, scaling dict or None, partial_rotary_factor) from either config.json flavour: the hub's
  top-level `rope_theta` + `rope_scaling`, or transformers-5's `rope_parameters` (theta inside)."""
  rp = cfg.get("rope_parameters") or {}
  theta = float(cfg.get("rope_theta", rp.get("rope_theta", 10000.0)))
  partial = float(cfg.get("partial_rotary_factor", rp.get("partial_rotary_factor", 1.0)) or 1.0)
  scaling = cfg.get("rope_scaling")
  if not scaling and rp:
    scaling = {k: v for k, v in rp.items() if k not in ("rope_theta", "partial_rotary_factor")}
  if scaling:
    kind = scaling.get("rope_type", scaling.get("type", "default"))
    if kind in ("su", "longrope"):  # Phi-3 LongRoPE: needs the pretraining window and the extended one
      scaling = dict(scaling, rope_type="longrope",
                     original_max_position_embeddings=int(scaling.get("original_max_position_embeddings")
                                                          or cfg.get("original_max_position_embeddings", 4096)),
                     max_position_embeddings=int(cfg.get("max_position_embeddings", 131072)))
    elif kind == "yarn":
      scaling = dict(scaling, rope_type="yarn",
                     original_max_position_embeddings=int(scaling.get("original_max_position_embeddings")
                                                          or cfg.get("original_max_position_embeddings", 4096)))
    elif kind in ("default", None):
      scaling = None
  return theta, (scaling or None), partial


def from_hf_config(cfg: dict) -> ModelConfig:
  mt = cfg.get("model_type", "llama")
  if mt == "llava":
    return _llava_config(cfg)
  H = int(cfg["num_attention_heads"])
  D = int(cfg["hidden_size"])
  eos = cfg.get("eos_token_id")
  eos_ids = tuple(eos) if isinstance(eos, (list, tuple)) else ((int(eos),) if eos is not None else (2,))
  theta, scaling, partial = _rope_fields(cfg)
  if cfg.get("sliding_window") and mt == "phi3":
    import warnings
    warnings.warn(f"phi3 sliding_window={cfg['sliding_window']} is not applied (full causal attention)")
  if mt in ("deepseek_v2", "deepseek_v3"):
    return _deepseek_config(cfg, mt, theta, scaling, eos_ids)
  return ModelConfig(
    model_type=mt,
    vocab_size=int(cfg["vocab_size"]),
    hidden_size=D,
    intermediate_size=int(cfg["intermediate_size"]),
    num_layers=int(cfg["num_hidden_layers"]),
    num_heads=H,
    num_kv_heads=int(cfg.get("num_key_value_heads", H)),
    head_dim=int(cfg.get("head_dim") or D // H),
    rms_norm_eps=float(cfg.get("rms_norm_eps", 1e-5)),
    rope_theta=theta,
    rope_scaling=scaling,
    max_position_embeddings=int(cfg.get("max_position_embeddings", 8192)),
    tie_word_embeddings=bool(cfg.get("tie_word_embeddings", False)),
    attention_bias=bool(cfg.get("attention_bias", mt == "qwen2")),
    num_experts=int(cfg.get("num_local_experts", 0)),
    num_experts_per_tok=int(cfg.get("num_experts_per_tok", 0)),
    bos_token_id=int(cfg.get("bos_token_id", 1) or 1),
    eos_token_ids=eos_ids,
    partial_rotary_factor=partial,
  )


def _deepseek_config(cfg: dict, mt: str, theta: float, scaling, eos_ids) -> ModelConfig:
  """DeepSeek-V2 / V3 (and R1): MLA attention, DeepSeekMoE with shared experts."""
  H = int(cfg["num_attention_heads"])
  v3 = mt == "deepseek_v3"
  return ModelConfig(
    model_type=mt,
    vocab_size=int(cfg["vocab_size"]),
    hidden_size=int(cfg["hidden_size"]),
    intermediate_size=int(cfg["intermediate_size"]),
    num_layers=int(cfg["num_hidden_layers"]),
    num_heads=H,
    num_kv_heads=1,  # one shared latent per token
    head_dim=int(cfg["qk_nope_head_dim"]) + int(cfg["qk_rope_head_dim"]),
    rms_norm_eps=float(cfg.get("rms_norm_eps", 1e-6)),
    rope_theta=theta,
    rope_scaling=scaling,
    max_position_embeddings=int(cfg.get("max_position_embeddings", 4096)),
    tie_word_embeddings=bool(cfg.get("tie_word_embeddings", False)),
    attention_bias=bool(cfg.get("attention_bias", False)),
    num_experts=int(cfg.get("n_routed_experts") or 0),
    num_experts_per_tok=int(cfg.get("num_experts_per_tok") or 0),
    bos_token_id=int(cfg.get("bos_token_id", 0) or 0),
    eos_token_ids=eos_ids,
    q_lora_rank=int(cfg.get("q_lora_rank") or 0),
    kv_lora_rank=int(cfg["kv_lora_rank"]),
    qk_nope_head_dim=int(cfg["qk_nope_head_dim"]),
    qk_rope_head_dim=int(cfg["qk_rope_head_dim"]),
    v_head_dim=int(cfg["v_head_dim"]),
    moe_intermediate_size=int(cfg.get("moe_intermediate_size") or 0),
    n_shared_experts=int(cfg.get("n_shared_experts") or 0),
    first_k_dense_replace=int(cfg.get("first_k_dense_replace") or 0),
    moe_layer_freq=int(cfg.get("moe_layer_freq") or 1),
    routed_scaling_factor=float(cfg.get("routed_scaling_factor") or 1.0),
    topk_method="noaux_tc" if v3 else str(cfg.get("topk_method") or "greedy"),
    n_group=int(cfg.get("n_group") or 1),
    topk_group=int(cfg.get("topk_group") or 1),
    # HF's V2 router never renormalises (norm_topk_prob is ignored there); V3 follows the flag
    norm_topk_prob=bool(cfg.get("norm_topk_prob", True)) if v3 else False,
    scoring_func="sigmoid" if v3 else "softmax",
  )


_VISION_KEYS = ("hidden_size", "intermediate_size", "num_hidden_layers", "num_attention_heads", "patch_size",
                "image_size", "layer_norm_eps", "hidden_act", "num_channels")


def _llava_config(cfg: dict) -> ModelConfig:
  """HF LlavaConfig: a Llama text model + CLIP vision tower (vision_config) + projector."""
  text = dict(cfg.get("text_config") or {})
  text.setdefault("model_type", "llama")
  for k in ("bos_token_id", "eos_token_id", "pad_token_id"):
    if k not in text and k in cfg:
      text[k] = cfg[k]
  lm = from_hf_config(text)
  vc = cfg.get("vision_config") or {}
  vision = {k: vc[k] for k in _VISION_KEYS if k in vc}
  vision.setdefault("num_channels", 3)
  vision.setdefault("hidden_act", "quick_gelu")
  vision.setdefault("layer_norm_eps", 1e-5)
  fl = cfg.get("vision_feature_layer", -2)
  if isinstance(fl, (list, tuple)):
    raise ValueError("multi-layer vision features are not supported")
  return replace(lm, model_type="llava", vision=vision,
                 image_token_id=int(cfg.get("image_token_index", cfg.get("image_token_id", 32000))),
                 vision_feature_layer=int(fl), vision_select=str(cfg.get("vision_feature_select_strategy", "default")),
                 projector_act=str(cfg.get("projector_hidden_act", "gelu")))


def load_config(model_dir: str | Path) -> ModelConfig:
  with open(Path(model_dir) / "config.json") as f:
    return from_hf_config(json.load(f))


_L3 = dict(rope_type="llama3", factor=32.0, low_freq_factor=1.0, high_freq_factor=4.0,
           original_max_position_embeddings=8192)
_L31 = dict(_L3, factor=8.0)
_DS_YARN = dict(rope_type="yarn", factor=40.0, original_max_position_embeddings=4096, beta_fast=32, beta_slow=1,
                mscale=1.0, mscale_all_dim=1.0)  # DeepSeek-V3 / R1
_DS2_YARN = dict(_DS_YARN, mscale=0.707, mscale_all_dim=0.707)  # DeepSeek-V2(-Lite)

PRESETS: dict[str, ModelConfig] = {
  "llama-3.2-1b": ModelConfig("llama", 128256, 2048, 8192, 16, 32, 8, 64, 1e-5, 500000.0, _L3, 131072, True),
  "llama-3.2-3b": ModelConfig("llama", 128256, 3072, 8192, 28, 24, 8, 128, 1e-5, 500000.0, _L3, 131072, True),
  "llama-3-8b": ModelConfig("llama", 128256, 4096, 14336, 32, 32, 8, 128, 1e-5, 500000.0, None, 8192, False),
  "llama-3.1-8b": ModelConfig("llama", 128256, 4096, 14336, 32, 32, 8, 128, 1e-5, 500000.0, _L31, 131072, False),
  "llama-3-70b": ModelConfig("llama", 128256, 8192, 28672, 80, 64, 8, 128, 1e-5, 500000.0, None, 8192, False),
  "llama-3.1-70b": ModelConfig("llama", 128256, 8192, 28672, 80, 64, 8, 128, 1e-5, 500000.0, _L31, 131072, False),
  "llama-3.3-70b": ModelConfig("llama", 128256, 8192, 28672, 80, 64, 8, 128, 1e-5, 500000.0, _L31, 131072, False),
  "qwen-2.5-0.5b": ModelConfig("qwen2", 151936, 896, 4864, 24, 14, 2, 64, 1e-6, 1000000.0, None, 32768, True, True,
                               bos_token_id=151643, eos_token_ids=(151645, 151643)),
  "qwen-2.5-1.5b": ModelConfig("qwen2", 151936, 1536, 8960, 28, 12, 2, 128, 1e-6, 1000000.0, None, 32768, True, True,
                               bos_token_id=151643, eos_token_ids=(151645, 151643)),
  "qwen-2.5-7b": ModelConfig("qwen2", 152064, 3584, 18944, 28, 28, 4, 128, 1e-6, 1000000.0, None, 32768, False, True,
                             bos_token_id=151643, eos_token_ids=(151645, 151643)),
  "qwen-2.5-3b": ModelConfig("qwen2", 151936, 2048, 11008, 36, 16, 2, 128, 1e-6, 1000000.0, None, 32768, True, True,
                             bos_token_id=151643, eos_token_ids=(151645, 151643)),
  "qwen-2.5-14b": ModelConfig("qwen2", 152064, 5120, 13824, 48, 40, 8, 128, 1e-5, 1000000.0, None, 32768, False, True,
                              bos_token_id=151643, eos_token_ids=(151645, 151643)),
  "qwen-2.5-32b": ModelConfig("qwen2", 152064, 5120, 27648, 64, 40, 8, 128, 1e-5, 1000000.0, None, 32768, False, True,
                              bos_token_id=151643, eos_token_ids=(151645, 151643)),
  "qwen-2.5-72b": ModelConfig("qwen2", 152064, 8192, 29568, 80, 64, 8, 128, 1e-5, 1000000.0, None, 32768, False, True,
                              bos_token_id=151643, eos_token_ids=(151645, 151643)),
  "llama-3.1-405b": ModelConfig("llama", 128256, 16384, 53248, 126, 128, 8, 128, 1e-5, 500000.0, _L31, 131072, False),
  "mistral-large": ModelConfig("mistral", 32768, 12288, 28672, 88, 96, 8, 128, 1e-5, 1000000.0, None, 131072, False,
                               bos_token_id=1, eos_token_ids=(2,)),
  "mistral-7b": ModelConfig("mistral", 32768, 4096, 14336, 32, 32, 8, 128, 1e-5, 1000000.0, None, 32768, False,
                            bos_token_id=1, eos_token_ids=(2,)),
  "mixtral-8x7b": ModelConfig("mixtral", 32000, 4096, 14336, 32, 32, 8, 128, 1e-5, 1000000.0, None, 32768, False,
                              num_experts=8, num_experts_per_tok=2, bos_token_id=1, eos_token_ids=(2,)),
  "mistral-nemo": ModelConfig("mistral", 131072, 5120, 14336, 40, 32, 8, 128, 1e-5, 1000000.0, None, 131072, False,
                              bos_token_id=1, eos_token_ids=(2,)),
  # Phi-4-mini (HF Phi3ForCausalLM): fused qkv / gate_up checkpoints, RoPE on 96 of 128 head dims, LongRoPE.
  # The hub config's 48 short / long LongRoPE factors are not available offline: the preset uses unit
  # factors (plain RoPE inside the 4k pretraining window, same attention factor); a downloaded config.json
  # carries the real ones.
  "phi-4-mini-instruct": ModelConfig("phi3", 200064, 3072, 8192, 32, 24, 8, 128, 1e-5, 10000.0,
                                     dict(rope_type="longrope", short_factor=[1.0] * 48, long_factor=[1.0] * 48,
                                          original_max_position_embeddings=4096, max_position_embeddings=131072),
                                     131072, True, bos_token_id=199999, eos_token_ids=(199999, 200020),
                                     partial_rotary_factor=0.75),
  # DeepSeek (HF DeepseekV2/V3ForCausalLM): MLA (latent 512 + rope 64), DeepSeekMoE with shared experts
  "deepseek-coder-v2-lite": ModelConfig("deepseek_v2", 102400, 2048, 10944, 27, 16, 1, 192, 1e-6, 10000.0,
                                        _DS2_YARN, 163840, False, num_experts=64, num_experts_per_tok=6,
                                        bos_token_id=100000, eos_token_ids=(100001,), kv_lora_rank=512,
                                        qk_nope_head_dim=128, qk_rope_head_dim=64, v_head_dim=128,
                                        moe_intermediate_size=1408, n_shared_experts=2, first_k_dense_replace=1,
                                        norm_topk_prob=False),
  "deepseek-v3": ModelConfig("deepseek_v3", 129280, 7168, 18432, 61, 128, 1, 192, 1e-6, 10000.0, _DS_YARN, 163840,
                             False, num_experts=256, num_experts_per_tok=8, bos_token_id=0, eos_token_ids=(1,),
                             q_lora_rank=1536, kv_lora_rank=512, qk_nope_head_dim=128, qk_rope_head_dim=64,
                             v_head_dim=128, moe_intermediate_size=2048, n_shared_experts=1, first_k_dense_replace=3,
                             routed_scaling_factor=2.5, topk_method="noaux_tc", n_group=8, topk_group=4,
                             norm_topk_prob=True, scoring_func="sigmoid"),
  # LLaVA-1.5-7B (HF LlavaForConditionalGeneration): Vicuna-7B text model + CLIP ViT-L/14-336 + MLP projector
  "llava-1.5-7b-hf": ModelConfig("llava", 32064, 4096, 11008, 32, 32, 32, 128, 1e-5, 10000.0, None, 4096, False,
                                 bos_token_id=1, eos_token_ids=(2,), image_token_id=32000,
                                 vision=dict(hidden_size=1024, intermediate_size=4096, num_hidden_layers=24,
                                             num_attention_heads=16, patch_size=14, image_size=336,
                                             layer_norm_eps=1e-5, hidden_act="quick_gelu", num_channels=3)),
  # small shapes for tests / CPU plumbing
  "tiny-llama": ModelConfig("llama", 512, 256, 512, 4, 4, 2, 64, 1e-5, 10000.0, None, 2048, False,
                            bos_token_id=1, eos_token_ids=(2,)),
  # 8 layers: multi-rank rehearsals of the 8-GPU ring (one layer per rank)
  "tiny-llama-8l": ModelConfig("llama", 512, 256, 512, 8, 4, 2, 64, 1e-5, 10000.0, None, 2048, False,
                               bos_token_id=1, eos_token_ids=(2,)),
  "tiny-llama-d64": ModelConfig("llama", 1024, 256, 512, 6, 4, 2, 64, 1e-5, 10000.0, _L3, 4096, True,
                                bos_token_id=1, eos_token_ids=(2,)),
  "tiny-qwen": ModelConfig("qwen2", 512, 256, 512, 4, 4, 2, 64, 1e-6, 1000000.0, None, 2048, True, True,
                           bos_token_id=1, eos_token_ids=(2,)),
  "tiny-mixtral": ModelConfig("mixtral", 512, 256, 512, 4, 4, 2, 64, 1e-5, 10000.0, None, 2048, False,
                              num_experts=4, num_experts_per_tok=2, bos_token_id=1, eos_token_ids=(2,)),
  "tiny-phi3": ModelConfig("phi3", 512, 256, 512, 4, 2, 1, 128, 1e-5, 10000.0,
                           dict(rope_type="longrope", short_factor=[1.0 + 0.05 * i for i in range(48)],
                                long_factor=[2.0 + 0.1 * i for i in range(48)], original_max_position_embeddings=64,
                                max_position_embeddings=2048), 2048, True, bos_token_id=1, eos_token_ids=(2,),
                           partial_rotary_factor=0.75),
  "tiny-llava": ModelConfig("llava", 512, 256, 512, 4, 4, 2, 64, 1e-5, 10000.0, None, 2048, False, bos_token_id=1,
                            eos_token_ids=(2,), image_token_id=500,
                            vision=dict(hidden_size=128, intermediate_size=256, num_hidden_layers=3, num_attention_heads=4,
                                        patch_size=14, image_size=56, layer_norm_eps=1e-5, hidden_act="quick_gelu",
                                        num_channels=3)),
  "tiny-deepseek-v2": ModelConfig("deepseek_v2", 512, 256, 512, 3, 4, 1, 192, 1e-6, 10000.0, None, 2048, False,
                                  num_experts=8, num_experts_per_tok=2, bos_token_id=1, eos_token_ids=(2,),
                                  kv_lora_rank=256, qk_nope_head_dim=128, qk_rope_head_dim=64, v_head_dim=128,
                                  moe_intermediate_size=256, n_shared_experts=2, first_k_dense_replace=1,
                                  topk_method="group_limited_greedy", n_group=4, topk_group=2, norm_topk_prob=False,
                                  routed_scaling_factor=1.5),
  "tiny-deepseek-v3": ModelConfig("deepseek_v3", 512, 256, 512, 3, 16, 1, 192, 1e-6, 10000.0,
                                  dict(_DS_YARN, original_max_position_embeddings=64), 2048, False, num_experts=16,
                                  num_experts_per_tok=4, bos_token_id=1, eos_token_ids=(2,), q_lora_rank=256,
                                  kv_lora_rank=256, qk_nope_head_dim=128, qk_rope_head_dim=64, v_head_dim=128,
                                  moe_intermediate_size=256, n_shared_experts=1, first_k_dense_replace=1,
                                  routed_scaling_factor=2.5, topk_method="noaux_tc", n_group=4, topk_group=2,
                                  norm_topk_prob=True, scoring_func="sigmoid"),
}
# aliases of the reference's model cards that share an architecture
for _alias, _base in {"llama-3.1-70b-bf16": "llama-3.1-70b", "nemotron-70b": "llama-3.1-70b",
                      "deepseek-r1-distill-llama-70b": "llama-3.1-70b", "deepseek-r1-distill-llama-8b": "llama-3.1-8b",
                      "qwen-2.5-coder-1.5b": "qwen-2.5-1.5b", "qwen-2.5-coder-7b": "qwen-2.5-7b",
                      "qwen-2.5-math-7b": "qwen-2.5-7b", "deepseek-r1-distill-qwen-1.5b": "qwen-2.5-1.5b",
                      "deepseek-r1-distill-qwen-7b": "qwen-2.5-7b", "qwen-2.5-coder-3b": "qwen-2.5-3b",
                      "qwen-2.5-coder-14b": "qwen-2.5-14b", "deepseek-r1-distill-qwen-14b": "qwen-2.5-14b",
                      "qwen-2.5-coder-32b": "qwen-2.5-32b", "deepseek-r1-distill-qwen-32b": "qwen-2.5-32b",
                      "qwen-2.5-math-72b": "qwen-2.5-72b", "llama-3.1-405b-8bit": "llama-3.1-405b",
                      "deepseek-r1": "deepseek-v3"}.items():
  PRESETS.setdefault(_alias, PRESETS[_base])


def preset(model_id: str) -> ModelConfig:
  if model_id not in PRESETS:
    raise KeyError(f"no built-in architecture preset for {model_id!r}; provide a config.json")
  return PRESETS[model_id]

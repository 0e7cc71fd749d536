"""Model cards: id -> layer count + HF repo per inference-engine class (reference: xotorch/models.py).

Same model ids as the reference (so clients and scripts keep working), plus the Mixtral MoE cards
this framework adds.  Layer counts follow the public HF configs; where the reference's card
disagrees (e.g. qwen-2.5-0.5b: 28 in the reference, 24 in config.json) the HF value is used and
`validate_layers` checks a downloaded config.json against the card.
"""
from __future__ import annotations

from typing import Dict, List, Optional

from ..inference.shard import Shard

ENGINE = "ShardedInferenceEngine"
DUMMY = "DummyInferenceEngine"

_CARDS: List[tuple] = [
  # id, layers, repo, pretty
  ("llama-3.3-70b", 80, "unsloth/Llama-3.3-70B-Instruct", "Llama 3.3 70B"),
  ("llama-3.2-1b", 16, "unsloth/Llama-3.2-1B-Instruct", "Llama 3.2 1B"),
  ("llama-3.2-3b", 28, "unsloth/Llama-3.2-3B-Instruct", "Llama 3.2 3B"),
  ("llama-3.1-8b", 32, "unsloth/Meta-Llama-3.1-8B-Instruct", "Llama 3.1 8B"),
  ("llama-3.1-70b", 80, "unsloth/Meta-Llama-3.1-70B-Instruct", "Llama 3.1 70B"),
  ("llama-3.1-70b-bf16", 80, "unsloth/Meta-Llama-3.1-70B-Instruct", "Llama 3.1 70B (BF16)"),
  ("llama-3-8b", 32, "unsloth/llama-3-8b", "Llama 3 8B"),
  ("llama-3-70b", 80, "unsloth/llama-3-70b", "Llama 3 70B"),
  ("llama-3.1-405b", 126, "unsloth/Meta-Llama-3.1-405B-Instruct-bnb-4bit", "Llama 3.1 405B"),
  ("llama-3.1-405b-8bit", 126, "unsloth/Meta-Llama-3.1-405B-Instruct-bnb-4bit", "Llama 3.1 405B (8-bit)"),
  ("mistral-nemo", 40, "unsloth/Mistral-Nemo-Instruct-2407-bnb-4bit", "Mistral Nemo"),
  ("mistral-large", 88, "unsloth/Mistral-Large-Instruct-2407-bnb-4bit", "Mistral Large"),
  ("mistral-7b", 32, "mistralai/Mistral-7B-Instruct-v0.3", "Mistral 7B"),
  ("mixtral-8x7b", 32, "mistralai/Mixtral-8x7B-Instruct-v0.1", "Mixtral 8x7B"),
  ("deepseek-coder-v2-lite", 27, "deepseek-ai/DeepSeek-Coder-V2-Lite-Instruct", "Deepseek Coder V2 Lite"),
  ("deepseek-v3", 61, "unsloth/DeepSeek-V3-bf16", "Deepseek V3"),
  ("deepseek-r1", 61, "deepseek-ai/DeepSeek-R1", "Deepseek R1"),
  ("deepseek-r1-distill-qwen-1.5b", 28, "unsloth/DeepSeek-R1-Distill-Qwen-1.5B", "DeepSeek R1 Distill Qwen 1.5B"),
  ("deepseek-r1-distill-qwen-7b", 28, "unsloth/DeepSeek-R1-Distill-Qwen-7B", "DeepSeek R1 Distill Qwen 7B"),
  ("deepseek-r1-distill-qwen-14b", 48, "unsloth/DeepSeek-R1-Distill-Qwen-14B", "DeepSeek R1 Distill Qwen 14B"),
  ("deepseek-r1-distill-qwen-32b", 64, "unsloth/DeepSeek-R1-Distill-Qwen-32B", "DeepSeek R1 Distill Qwen 32B"),
  ("deepseek-r1-distill-llama-8b", 32, "unsloth/DeepSeek-R1-Distill-Llama-8B", "DeepSeek R1 Distill Llama 8B"),
  ("deepseek-r1-distill-llama-70b", 80, "unsloth/DeepSeek-R1-Distill-Llama-70B", "DeepSeek R1 Distill Llama 70B"),
  ("llava-1.5-7b-hf", 32, "llava-hf/llava-1.5-7b-hf", "LLaVa 1.5 7B (Vision Model)"),
  ("qwen-2.5-0.5b", 24, "unsloth/Qwen2.5-0.5B-Instruct", "Qwen 2.5 0.5B"),
  ("qwen-2.5-1.5b", 28, "unsloth/Qwen2.5-1.5B-Instruct", "Qwen 2.5 1.5B"),
  ("qwen-2.5-coder-1.5b", 28, "unsloth/Qwen2.5-Coder-1.5B-Instruct", "Qwen 2.5 Coder 1.5B"),
  ("qwen-2.5-3b", 36, "unsloth/Qwen2.5-3B-Instruct", "Qwen 2.5 3B"),
  ("qwen-2.5-coder-3b", 36, "unsloth/Qwen2.5-Coder-3B-Instruct", "Qwen 2.5 Coder 3B"),
  ("qwen-2.5-7b", 28, "unsloth/Qwen2.5-7B-Instruct", "Qwen 2.5 7B"),
  ("qwen-2.5-coder-7b", 28, "unsloth/Qwen2.5-Coder-7B-Instruct", "Qwen 2.5 Coder 7B"),
  ("qwen-2.5-math-7b", 28, "Qwen/Qwen2.5-Math-7B-Instruct", "Qwen 2.5 7B (Math)"),
  ("qwen-2.5-14b", 48, "unsloth/Qwen2.5-14B-Instruct", "Qwen 2.5 14B"),
  ("qwen-2.5-coder-14b", 48, "unsloth/Qwen2.5-Coder-14B-Instruct", "Qwen 2.5 Coder 14B"),
  ("qwen-2.5-32b", 64, "Qwen/Qwen2.5-32B-Instruct", "Qwen 2.5 32B"),
  ("qwen-2.5-coder-32b", 64, "Qwen/Qwen2.5-Coder-32B-Instruct", "Qwen 2.5 Coder 32B"),
  ("qwen-2.5-72b", 80, "Qwen/Qwen2.5-72B-Instruct", "Qwen 2.5 72B"),
  ("qwen-2.5-math-72b", 80, "Qwen/Qwen2.5-Math-72B-Instruct", "Qwen 2.5 72B (Math)"),
  ("nemotron-70b", 80, "nvidia/Llama-3.1-Nemotron-70B-Instruct-HF", "Nemotron 70B"),
  ("phi-4-mini-instruct", 32, "microsoft/Phi-4-mini-instruct", "Phi-4 Mini Instruct"),
  # synthetic architectures (random init, no download) for tests and the offline GPU box
  ("tiny-llama", 4, "synthetic/tiny-llama", "Tiny Llama (synthetic)"),
  ("tiny-llama-d64", 6, "synthetic/tiny-llama-d64", "Tiny Llama d64 (synthetic)"),
  ("tiny-qwen", 4, "synthetic/tiny-qwen", "Tiny Qwen (synthetic)"),
  ("tiny-mixtral", 4, "synthetic/tiny-mixtral", "Tiny Mixtral (synthetic)"),
  ("tiny-phi3", 4, "synthetic/tiny-phi3", "Tiny Phi-3 (synthetic)"),
  ("tiny-deepseek-v2", 3, "synthetic/tiny-deepseek-v2", "Tiny DeepSeek-V2 (synthetic)"),
  ("tiny-deepseek-v3", 3, "synthetic/tiny-deepseek-v3", "Tiny DeepSeek-V3 (synthetic)"),
  ("tiny-llava", 4, "synthetic/tiny-llava", "Tiny LLaVA (synthetic)"),
]

model_cards: Dict[str, dict] = {mid: {"layers": n, "repo": {ENGINE: repo}} for mid, n, repo, _ in _CARDS}
SYNTHETIC = {mid for mid, _, repo, _ in _CARDS if repo.startswith("synthetic/")}
model_cards["dummy"] = {"layers": 8, "repo": {DUMMY: "dummy"}}
pretty_name: Dict[str, str] = {mid: pretty for mid, _, _, pretty in _CARDS}
pretty_name["dummy"] = "Dummy"


def get_repo(model_id: str, engine_classname: str) -> Optional[str]:
  return model_cards.get(model_id, {}).get("repo", {}).get(engine_classname)


def get_pretty_name(model_id: str) -> Optional[str]:
  return pretty_name.get(model_id)


def build_base_shard(model_id: str, engine_classname: str) -> Optional[Shard]:
  if get_repo(model_id, engine_classname) is None:
    return None
  n = int(model_cards[model_id].get("layers", 0))
  return Shard(model_id, 0, 0, n) if n > 0 else None


def build_full_shard(model_id: str, engine_classname: str) -> Optional[Shard]:
  base = build_base_shard(model_id, engine_classname)
  return None if base is None else Shard(model_id, 0, base.n_layers - 1, base.n_layers)


def get_supported_models(engine_lists: Optional[List[List[str]]] = None) -> List[str]:
  """Models that every peer can run: each inner list is one peer's engines (names or class names)."""
  if not engine_lists:
    return list(model_cards)
  from ..inference.inference_engine import inference_engine_classes
  lists = [[inference_engine_classes.get(e, e) for e in lst] for lst in engine_lists]
  return [mid for mid, card in model_cards.items() if all(any(e in card["repo"] for e in lst) for lst in lists)]


def validate_layers(model_id: str, config_layers: int) -> int:
  """Return the authoritative layer count (config.json) and warn on a card mismatch."""
  card = model_cards.get(model_id, {}).get("layers")
  if card is not None and card != config_layers:
    import warnings
    warnings.warn(f"model card {model_id} says {card} layers but config.json has {config_layers}; using config.json")
  return config_layers


def is_vision_model(model_id: str) -> bool:
  """Cards whose architecture has an image tower (LLaVA): the API keeps their images."""
  from .config import PRESETS
  c = PRESETS.get(model_id)
  return bool(c is not None and c.vision) or "llava" in model_id

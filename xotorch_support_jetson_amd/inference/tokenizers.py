"""Tokenizer resolution (reference: xotorch/inference/tokenizers.py:11-63).

Prefers a local model directory (downloaded shard), then the HF hub cache (offline), and finally —
this framework runs on boxes with no network — a built-in byte-level tokenizer with a chat template,
so the CLI / API / ring work end to end on random-init weights.
"""
from __future__ import annotations

import os
from pathlib import Path
from typing import List, Optional, Union

import numpy as np

from ..helpers import DEBUG


class DummyTokenizer:
  def __init__(self):
    self.eos_token_id = 69
    self.vocab_size = 1000

  def apply_chat_template(self, conversation, tokenize=True, add_generation_prompt=True, tools=None, **kwargs):
    return "dummy_tokenized_prompt"

  def encode(self, text, **kwargs):
    return [1]

  def decode(self, tokens, **kwargs):
    return "dummy" * len(tokens)


class ByteTokenizer:
  """UTF-8 bytes -> ids [3, 259); 0 pad, 1 bos, 2 eos.  Ids >= 259 (a real model's larger vocab)
  decode to nothing, so random-weight generations stay printable."""

  def __init__(self, vocab_size: int = 259, bos_token_id: int = 1, eos_token_id: int = 2):
    self.vocab_size = max(vocab_size, 259)
    self.bos_token_id = bos_token_id
    self.eos_token_id = eos_token_id
    self.pad_token_id = 0
    self.chat_template = "byte"

  def encode(self, text: str, add_special_tokens: bool = True, **kwargs) -> List[int]:
    ids = [b + 3 for b in text.encode("utf-8")]
    return ([self.bos_token_id] + ids) if add_special_tokens else ids

  def decode(self, tokens, skip_special_tokens: bool = True, **kwargs) -> str:
    if isinstance(tokens, np.ndarray):
      tokens = tokens.reshape(-1).tolist()
    out = bytes(int(t) - 3 for t in tokens if 3 <= int(t) < 259)
    return out.decode("utf-8", errors="replace")

  def apply_chat_template(self, messages, tokenize: bool = False, add_generation_prompt: bool = True, tools=None,
                          **kwargs) -> Union[str, List[int]]:
    parts = []
    for m in messages:
      content = m["content"] if isinstance(m, dict) else getattr(m, "content", "")
      if isinstance(content, list):
        content = "".join(c.get("text", "") for c in content if isinstance(c, dict))
      role = m["role"] if isinstance(m, dict) else getattr(m, "role", "user")
      parts.append(f"<|{role}|>\n{content}\n")
    if add_generation_prompt:
      parts.append("<|assistant|>\n")
    text = "".join(parts)
    return self.encode(text) if tokenize else text


def _local_candidates(repo_id: str) -> List[Path]:
  from ..helpers import xot_home
  cands = [xot_home() / "downloads" / repo_id.replace("/", "--")]
  hf = Path(os.environ.get("HF_HOME", Path.home() / ".cache" / "huggingface")) / "hub"
  snap = hf / f"models--{repo_id.replace('/', '--')}" / "snapshots"
  if snap.exists():
    cands += sorted(snap.iterdir())
  return cands


async def resolve_tokenizer(repo_id: Union[str, Path], vocab_size: Optional[int] = None):
  return _resolve_tokenizer(repo_id, vocab_size)


def _resolve_tokenizer(repo_id: Union[str, Path], vocab_size: Optional[int] = None):
  if str(repo_id) == "dummy":
    return DummyTokenizer()
  paths = [Path(repo_id)] if Path(str(repo_id)).exists() else _local_candidates(str(repo_id))
  for p in paths:
    if (p / "tokenizer.json").exists() or (p / "tokenizer_config.json").exists():
      try:
        from transformers import AutoTokenizer
        tok = AutoTokenizer.from_pretrained(str(p), trust_remote_code=False)
        return tok
      except Exception as e:  # pragma: no cover - depends on local files
        if DEBUG >= 1:
          print(f"tokenizer load failed from {p}: {e}")
  if DEBUG >= 1:
    print(f"no local tokenizer for {repo_id}; using the built-in byte tokenizer (offline)")
  return ByteTokenizer(vocab_size or 259)

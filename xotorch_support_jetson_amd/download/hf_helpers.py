"""HF hub helpers: endpoint, auth token and allow-pattern filtering (reference: xotorch/download/hf/hf_helpers.py)."""
from __future__ import annotations

import fnmatch
import os
from pathlib import Path
from typing import Callable, Dict, Generator, Iterable, List, Optional, TypeVar, Union

from ..inference.shard import Shard

T = TypeVar("T")

ALWAYS = ["*.json", "*.py", "tokenizer.model", "tiktoken.model", "*.tiktoken", "*.txt", "*.jinja"]


def get_hf_endpoint() -> str:
  return os.environ.get("HF_ENDPOINT", "https://huggingface.co").rstrip("/")


def get_hf_home() -> Path:
  return Path(os.environ.get("HF_HOME", Path.home() / ".cache" / "huggingface"))


def get_hf_token() -> Optional[str]:
  tok = os.environ.get("HF_TOKEN")
  if tok:
    return tok
  p = get_hf_home() / "token"
  try:
    return p.read_text().strip() or None
  except OSError:
    return None


def get_auth_headers() -> Dict[str, str]:
  tok = get_hf_token()
  return {"Authorization": f"Bearer {tok}"} if tok else {}


def filter_repo_objects(items: Iterable[T], allow_patterns: Optional[Union[List[str], str]] = None,
                        ignore_patterns: Optional[Union[List[str], str]] = None,
                        key: Optional[Callable[[T], str]] = None) -> Generator[T, None, None]:
  if isinstance(allow_patterns, str):
    allow_patterns = [allow_patterns]
  if isinstance(ignore_patterns, str):
    ignore_patterns = [ignore_patterns]

  def norm(p: str) -> str:
    return p + "*" if p.endswith("/") else p

  allow = [norm(p) for p in allow_patterns] if allow_patterns else None
  ignore = [norm(p) for p in ignore_patterns] if ignore_patterns else None
  for item in items:
    path = key(item) if key else item
    if allow is not None and not any(fnmatch.fnmatch(path, p) for p in allow):
      continue
    if ignore is not None and any(fnmatch.fnmatch(path, p) for p in ignore):
      continue
    yield item


def get_allow_patterns(weight_map: Dict[str, str], shard: Shard) -> List[str]:
  """Config/tokenizer files + only the safetensors files holding this shard's tensors."""
  files = set()
  for name, fname in weight_map.items():
    if name.startswith("model.layers."):
      try:
        layer = int(name.split(".")[2])
      except (IndexError, ValueError):
        continue
      if shard.start_layer <= layer <= shard.end_layer:
        files.add(fname)
    elif name.startswith("model.embed_tokens") and (shard.is_first_layer() or shard.is_last_layer()):
      files.add(fname)
    elif (name.startswith("model.norm") or name.startswith("lm_head")) and shard.is_last_layer():
      files.add(fname)
  return ALWAYS + sorted(files)

"""Deterministic fake backend for plumbing tests (reference: xotorch/inference/dummy_inference_engine.py).

Last shard returns input + 1; other shards pass through.  `sample` returns the input until it exceeds
10, then the EOS id 69 — so a ring of dummy peers generates [2, 3, ..., 10, 69] for any prompt.
"""
from __future__ import annotations

import asyncio
from typing import Optional, Tuple

import numpy as np

from .inference_engine import InferenceEngine
from .shard import Shard
from .tokenizers import DummyTokenizer


class DummyInferenceEngine(InferenceEngine):
  def __init__(self):
    self.shard: Optional[Shard] = None
    self.vocab_size = 1000
    self.hidden_size = 256
    self.eos_token_id = 69
    self.latency_mean = 0.0
    self.tokenizer = DummyTokenizer()
    self.trained = []
    self.saved = []

  async def encode(self, shard: Shard, prompt: str) -> np.ndarray:
    return np.array(self.tokenizer.encode(prompt))

  async def sample(self, x: np.ndarray, temp: float = 0.0, top_k: int = 35) -> np.ndarray:
    if x[0] > 10:
      return np.array([self.eos_token_id])
    return x

  async def decode(self, shard: Shard, tokens: np.ndarray) -> str:
    return self.tokenizer.decode(tokens)

  async def infer_tensor(self, request_id: str, shard: Shard, input_data: np.ndarray,
                         inference_state: Optional[dict] = None) -> Tuple[np.ndarray, Optional[dict]]:
    await self.ensure_shard(shard)
    if self.latency_mean:
      await asyncio.sleep(self.latency_mean)
    return (input_data + 1 if self.shard.is_last_layer() else input_data), None

  async def ensure_shard(self, shard: Shard):
    self.shard = shard

  async def load_checkpoint(self, shard: Shard, path: str):
    await self.ensure_shard(shard)

  async def save_checkpoint(self, shard: Shard, path: str):
    self.saved.append((shard, path))

  async def train(self, request_id, shard, example, target, length, train=True, loss="length_masked_ce"):
    await self.ensure_shard(shard)
    self.trained.append(request_id)
    grad = np.zeros_like(example, dtype=np.float32) if not shard.is_first_layer() else None
    return 1.0, grad

  async def evaluate(self, request_id, shard, example, target, length, loss="length_masked_ce"):
    await self.ensure_shard(shard)
    return 1.0

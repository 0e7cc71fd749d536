"""Inference-engine contract used by the Node (reference: xotorch/inference/inference_engine.py:11-70).

Same async surface as the reference (encode / sample / decode / infer_tensor / infer_prompt /
load_checkpoint / save_checkpoint) plus the training hooks the reference's Node calls but never
implements (train / evaluate, node.py:299-345) and `finish_request` to release a request's KV pages.
"""
from __future__ import annotations

from abc import ABC, abstractmethod
from typing import Optional, Tuple

import numpy as np

from ..helpers import DEBUG
from .shard import Shard


class InferenceEngine(ABC):
  session: dict = {}

  @abstractmethod
  async def encode(self, shard: Shard, prompt: str) -> np.ndarray:
    ...

  @abstractmethod
  async def sample(self, x: np.ndarray, temp: float = 0.0, top_k: int = 35) -> np.ndarray:
    ...

  @abstractmethod
  async def decode(self, shard: Shard, tokens: np.ndarray) -> str:
    ...

  @abstractmethod
  async def infer_tensor(self, request_id: str, shard: Shard, input_data: np.ndarray,
                         inference_state: Optional[dict] = None) -> Tuple[np.ndarray, Optional[dict]]:
    ...

  @abstractmethod
  async def load_checkpoint(self, shard: Shard, path: str):
    ...

  async def save_checkpoint(self, shard: Shard, path: str):
    raise NotImplementedError(f"{type(self).__name__} cannot save checkpoints")

  async def train(self, request_id: str, shard: Shard, example, target, length, train: bool = True,
                  loss: str = "length_masked_ce"):
    raise NotImplementedError(f"{type(self).__name__} does not train")

  async def evaluate(self, request_id: str, shard: Shard, example, target, length, loss: str = "length_masked_ce"):
    raise NotImplementedError(f"{type(self).__name__} does not evaluate")

  async def finish_request(self, request_id: str, ok: bool = True) -> None:
    """Release per-request state (KV pages).  Called when a generation ends; ok=False when it failed or
    was aborted part-way (its steps may not have reached every shard)."""

  async def save_session(self, key, value):
    self.session[key] = value

  async def clear_session(self):
    self.session.clear()

  async def infer_prompt(self, request_id: str, shard: Shard, prompt: str,
                         inference_state: Optional[dict] = None) -> Tuple[np.ndarray, Optional[dict]]:
    tokens = await self.encode(shard, prompt)
    return await self.infer_tensor(request_id, shard, tokens.reshape(1, -1), inference_state)


# CLI name -> engine class name (model cards key their repos by class name)
inference_engine_classes = {
  "mi355x": "ShardedInferenceEngine",
  "torch": "ShardedInferenceEngine",  # the reference's default engine name keeps working
  "dummy": "DummyInferenceEngine",
}


def get_inference_engine(inference_engine_name: str, shard_downloader):
  if DEBUG >= 2:
    print(f"get_inference_engine called with: {inference_engine_name}")
  if inference_engine_name in ("mi355x", "torch"):
    from .sharded_engine import ShardedInferenceEngine
    return ShardedInferenceEngine(shard_downloader)
  if inference_engine_name == "dummy":
    from .dummy_inference_engine import DummyInferenceEngine
    return DummyInferenceEngine()
  raise ValueError(f"Unsupported inference engine: {inference_engine_name}")

"""Shard downloader contract + no-op implementation (reference: xotorch/download/shard_download.py)."""
from __future__ import annotations

from abc import ABC, abstractmethod
from pathlib import Path
from typing import AsyncIterator, Optional, Tuple

from ..helpers import AsyncCallbackSystem
from ..inference.shard import Shard
from .download_progress import RepoProgressEvent


class ShardDownloader(ABC):
  @abstractmethod
  async def ensure_shard(self, shard: Shard, inference_engine_name: str) -> Path:
    """Make the files this shard needs available locally; returns the model directory."""

  @property
  @abstractmethod
  def on_progress(self) -> AsyncCallbackSystem[str, Tuple[Shard, RepoProgressEvent]]:
    ...

  @abstractmethod
  async def get_shard_download_status(self, inference_engine_name: str) -> AsyncIterator[Tuple[Path, RepoProgressEvent]]:
    ...


class NoopShardDownloader(ShardDownloader):
  def __init__(self):
    self._on_progress = AsyncCallbackSystem[str, Tuple[Shard, RepoProgressEvent]]()

  async def ensure_shard(self, shard: Shard, inference_engine_name: str) -> Optional[Path]:
    return None

  @property
  def on_progress(self):
    return self._on_progress

  async def get_shard_download_status(self, inference_engine_name: str):
    if False:  # pragma: no cover - async generator with no items
      yield

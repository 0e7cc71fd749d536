"""Peer handle contract (reference: xotorch/networking/peer_handle.py:9-56)."""
from __future__ import annotations

from abc import ABC, abstractmethod
from typing import Optional

import numpy as np

from ..inference.shard import Shard
from ..topology.device_capabilities import DeviceCapabilities
from ..topology.topology import Topology


class PeerHandle(ABC):
  @abstractmethod
  def id(self) -> str: ...

  @abstractmethod
  def addr(self) -> str: ...

  @abstractmethod
  def description(self) -> str: ...

  @abstractmethod
  def device_capabilities(self) -> DeviceCapabilities: ...

  @abstractmethod
  async def connect(self) -> None: ...

  @abstractmethod
  async def is_connected(self) -> bool: ...

  @abstractmethod
  async def disconnect(self) -> None: ...

  @abstractmethod
  async def health_check(self) -> bool: ...

  @abstractmethod
  async def send_prompt(self, shard: Shard, prompt: str, request_id: Optional[str] = None,
                        inference_state: Optional[dict] = None) -> None: ...

  @abstractmethod
  async def send_tensor(self, shard: Shard, tensor, request_id: Optional[str] = None,
                        inference_state: Optional[dict] = None) -> None: ...

  @abstractmethod
  async def send_example(self, shard: Shard, example, target, length, train: bool,
                         request_id: Optional[str] = None): ...

  @abstractmethod
  async def send_result(self, request_id: str, result, is_finished: bool) -> None: ...

  @abstractmethod
  async def send_opaque_status(self, request_id: str, status: str) -> None: ...

  @abstractmethod
  async def collect_topology(self, visited: set, max_depth: int) -> Topology: ...

"""Manual discovery from a JSON topology file (reference: xotorch/networking/manual/manual_discovery.py).

Re-reads the file whenever its mtime changes, polls every `poll_interval` seconds, keeps only peers
that pass a health check.  The node's own id must be present in the file.
"""
from __future__ import annotations

import asyncio
import os
from typing import Callable, Dict, List, Optional

from ...helpers import DEBUG_DISCOVERY
from ...topology.device_capabilities import DeviceCapabilities
from ..discovery import Discovery
from ..peer_handle import PeerHandle
from .network_topology_config import NetworkTopology, PeerConfig


class ManualDiscovery(Discovery):
  def __init__(self, network_config_path: str, node_id: str,
               create_peer_handle: Callable[[str, str, str, DeviceCapabilities], PeerHandle],
               poll_interval: float = 5.0):
    self.network_config_path = network_config_path
    self.node_id = node_id
    self.create_peer_handle = create_peer_handle
    self.poll_interval = poll_interval
    self.known_peers: Dict[str, PeerHandle] = {}
    self._task: Optional[asyncio.Task] = None
    self._cached: Optional[Dict[str, PeerConfig]] = None
    self._mtime = 0.0

  async def start(self) -> None:
    self._task = asyncio.create_task(self.task_find_peers_from_config())

  async def stop(self) -> None:
    if self._task:
      self._task.cancel()
      await asyncio.gather(self._task, return_exceptions=True)

  async def discover_peers(self, wait_for_peers: int = 0) -> List[PeerHandle]:
    if wait_for_peers > 0:
      while len(self.known_peers) < wait_for_peers:
        await asyncio.sleep(0.1)
    return list(self.known_peers.values())

  async def refresh(self) -> None:
    peers = self._get_peers()
    alive: Dict[str, PeerHandle] = {}
    for pid, cfg in peers.items():
      addr = f"{cfg.address}:{cfg.port}"
      handle = self.known_peers.get(pid)
      if handle is None or handle.addr() != addr:
        handle = self.create_peer_handle(pid, addr, "MAN", cfg.device_capabilities)
      try:
        healthy = await handle.health_check()
      except Exception:
        healthy = False
      if healthy:
        alive[pid] = handle
      elif DEBUG_DISCOVERY >= 1:
        print(f"manual peer {pid} at {addr} is not healthy")
    self.known_peers = alive

  async def task_find_peers_from_config(self):
    while True:
      try:
        await self.refresh()
      except Exception as e:
        if DEBUG_DISCOVERY >= 1:
          print(f"manual discovery error: {e}")
      await asyncio.sleep(self.poll_interval)

  def _get_peers(self) -> Dict[str, PeerConfig]:
    mtime = os.path.getmtime(self.network_config_path)
    if self._cached is None or mtime != self._mtime:
      topo = NetworkTopology.from_path(self.network_config_path)
      if self.node_id not in topo.peers:
        raise ValueError(f"node id {self.node_id} not found in {self.network_config_path}")
      self._cached = {pid: cfg for pid, cfg in topo.peers.items() if pid != self.node_id}
      self._mtime = mtime
    return self._cached

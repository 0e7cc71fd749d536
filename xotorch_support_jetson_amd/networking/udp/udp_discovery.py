"""UDP broadcast discovery (reference: xotorch/networking/udp/udp_discovery.py:13-246).

Every `broadcast_interval` s each node broadcasts a JSON presence datagram
{type: "discovery", node_id, grpc_port, device_capabilities, priority, interface_name, interface_type}
on every IPv4 interface (subnet broadcast + 255.255.255.255).  A listener keeps, per peer, the
highest-priority interface it was heard on, health-checks it over gRPC and drops peers that fail a
health check or stay silent for `discovery_timeout` seconds.  Allow-lists by node id / interface type.
"""
from __future__ import annotations

import asyncio
import json
import socket
import time
import traceback
from typing import Callable, Dict, List, Optional, Tuple

from ...helpers import DEBUG_DISCOVERY, get_all_ip_addresses_and_interfaces, get_broadcast_address, \
  get_interface_priority_and_type
from ...topology.device_capabilities import DeviceCapabilities, device_capabilities
from ..discovery import Discovery
from ..peer_handle import PeerHandle


class _Listen(asyncio.DatagramProtocol):
  def __init__(self, on_message: Callable):
    self.on_message = on_message

  def datagram_received(self, data, addr):
    asyncio.create_task(self.on_message(data, addr))


class _Broadcast(asyncio.DatagramProtocol):
  def __init__(self, message: str, broadcast_port: int, source_ip: str):
    self.message = message
    self.broadcast_port = broadcast_port
    self.source_ip = source_ip

  def connection_made(self, transport):
    sock = transport.get_extra_info("socket")
    sock.setsockopt(socket.SOL_SOCKET, socket.SO_BROADCAST, 1)
    for target in {get_broadcast_address(self.source_ip), "255.255.255.255"}:
      try:
        transport.sendto(self.message.encode("utf-8"), (target, self.broadcast_port))
      except OSError:
        pass


class UDPDiscovery(Discovery):
  def __init__(self, node_id: str, node_port: int, listen_port: int, broadcast_port: int,
               create_peer_handle: Callable[[str, str, str, DeviceCapabilities], PeerHandle],
               broadcast_interval: float = 2.5, discovery_timeout: float = 30,
               device_capabilities_override: Optional[DeviceCapabilities] = None,
               allowed_node_ids: Optional[List[str]] = None, allowed_interface_types: Optional[List[str]] = None):
    self.node_id = node_id
    self.node_port = node_port
    self.listen_port = listen_port
    self.broadcast_port = broadcast_port
    self.create_peer_handle = create_peer_handle
    self.broadcast_interval = broadcast_interval
    self.discovery_timeout = discovery_timeout
    self.device_capabilities = device_capabilities_override
    self.allowed_node_ids = allowed_node_ids
    self.allowed_interface_types = allowed_interface_types
    # peer_id -> (handle, connected_at, last_seen, priority)
    self.known_peers: Dict[str, Tuple[PeerHandle, float, float, int]] = {}
    self.tasks: List[asyncio.Task] = []
    self.listen_transport = None

  async def start(self):
    if self.device_capabilities is None:
      self.device_capabilities = device_capabilities()
    self.tasks = [asyncio.create_task(self.task_broadcast_presence()),
                  asyncio.create_task(self.task_listen_for_peers()),
                  asyncio.create_task(self.task_cleanup_peers())]

  async def stop(self):
    for t in self.tasks:
      t.cancel()
    await asyncio.gather(*self.tasks, return_exceptions=True)
    if self.listen_transport:
      self.listen_transport.close()

  async def discover_peers(self, wait_for_peers: int = 0) -> List[PeerHandle]:
    if wait_for_peers > 0:
      while len(self.known_peers) < wait_for_peers:
        if DEBUG_DISCOVERY >= 2:
          print(f"waiting for peers: {len(self.known_peers)}/{wait_for_peers}")
        await asyncio.sleep(0.1)
    return [p for p, _, _, _ in self.known_peers.values()]

  # ------------------------------------------------------------------ tasks
  async def task_broadcast_presence(self):
    while True:
      for ip, ifname in get_all_ip_addresses_and_interfaces():
        prio, kind = get_interface_priority_and_type(ifname)
        msg = json.dumps({"type": "discovery", "node_id": self.node_id, "grpc_port": self.node_port,
                          "device_capabilities": self.device_capabilities.to_dict(), "priority": prio,
                          "interface_name": ifname, "interface_type": kind})
        transport = None
        try:
          transport, _ = await asyncio.get_running_loop().create_datagram_endpoint(
            lambda: _Broadcast(msg, self.broadcast_port, ip), local_addr=(ip, 0), family=socket.AF_INET)
        except Exception as e:
          if DEBUG_DISCOVERY >= 2:
            print(f"broadcast on {ip} ({ifname}) failed: {e}")
        finally:
          if transport:
            transport.close()
      await asyncio.sleep(self.broadcast_interval)

  async def task_listen_for_peers(self):
    loop = asyncio.get_running_loop()
    sock = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    try:
      sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEPORT, 1)
    except (AttributeError, OSError):
      pass
    sock.bind(("", self.listen_port))
    self.listen_transport, _ = await loop.create_datagram_endpoint(lambda: _Listen(self.on_listen_message), sock=sock)
    if DEBUG_DISCOVERY >= 2:
      print(f"listening for peers on port {self.listen_port}")

  async def on_listen_message(self, data: bytes, addr):
    if not data:
      return
    try:
      msg = json.loads(data.decode("utf-8", errors="ignore"))
    except json.JSONDecodeError:
      return
    if msg.get("type") != "discovery" or msg.get("node_id") == self.node_id:
      return
    peer_id = msg["node_id"]
    if self.allowed_node_ids and peer_id not in self.allowed_node_ids:
      return
    kind = msg.get("interface_type", "Other")
    if self.allowed_interface_types and kind not in self.allowed_interface_types:
      return
    peer_host = addr[0]
    peer_port = msg["grpc_port"]
    prio = int(msg.get("priority", 1))
    caps = DeviceCapabilities(**msg["device_capabilities"])
    now = time.time()
    known = self.known_peers.get(peer_id)
    addr_str = f"{peer_host}:{peer_port}"
    better = known is None or prio > known[3] or (known[0].addr() != addr_str and prio >= known[3])
    if better:
      handle = self.create_peer_handle(peer_id, f"{peer_host}:{peer_port}", f"{kind} ({msg.get('interface_name')})",
                                       caps)
      if not await handle.health_check():
        if DEBUG_DISCOVERY >= 1:
          print(f"peer {peer_id} at {peer_host}:{peer_port} failed its health check")
        return
      self.known_peers[peer_id] = (handle, now, now, prio)
      if DEBUG_DISCOVERY >= 1:
        print(f"discovered peer {peer_id} at {peer_host}:{peer_port} ({kind})")
    else:
      self.known_peers[peer_id] = (known[0], known[1], now, known[3])

  async def task_cleanup_peers(self):
    while True:
      try:
        now = time.time()
        for pid, (handle, connected_at, last_seen, prio) in list(self.known_peers.items()):
          stale = now - last_seen > self.discovery_timeout
          healthy = await handle.health_check() if not stale else False
          if stale or not healthy:
            if DEBUG_DISCOVERY >= 1:
              print(f"removing peer {pid} (stale={stale}, healthy={healthy})")
            self.known_peers.pop(pid, None)
      except Exception:
        if DEBUG_DISCOVERY >= 1:
          traceback.print_exc()
      await asyncio.sleep(self.broadcast_interval)

"""Cross-cutting runtime utilities (reference: xotorch/helpers.py).

DEBUG levels, the async event bus used for tokens / status / download progress, free-port
selection, persistent node id, network-interface ranking and graceful shutdown.
"""
from __future__ import annotations

import asyncio
import os
import random
import signal
import socket
import tempfile
import uuid
from pathlib import Path
from typing import Any, Callable, Dict, Generic, List, Optional, Tuple, TypeVar

import psutil

DEBUG = int(os.getenv("DEBUG", "0"))
DEBUG_DISCOVERY = int(os.getenv("DEBUG_DISCOVERY", "0"))
VERSION = "0.1.0"

XOT_BANNER = r"""
 __  __  ___  _____
 \ \/ / / _ \|_   _|
  >  < | (_) | | |    MI355X
 /_/\_\ \___/  |_|
"""

T = TypeVar("T")
K = TypeVar("K")


def print_banner(color: bool = False) -> None:
  print(f"\x1b[31m{XOT_BANNER}\x1b[0m" if color else XOT_BANNER)


def terminal_link(uri: str, label: Optional[str] = None) -> str:
  return f"\033]8;;{uri}\033\\{label or uri}\033]8;;\033\\"


# ------------------------------------------------------------------ event bus
class AsyncCallback(Generic[T]):
  """Latest-value slot with observers and an awaitable predicate wait."""

  def __init__(self) -> None:
    self._cond = asyncio.Condition()
    self.result: Optional[Tuple[T, ...]] = None
    self.observers: List[Callable[..., Any]] = []
    self._waiters = 0  # coroutines inside wait(): set() schedules a notify only for them

  async def wait(self, predicate: Callable[..., bool], timeout: Optional[float] = None) -> Tuple[T, ...]:
    self._waiters += 1
    try:
      async with self._cond:
        await asyncio.wait_for(self._cond.wait_for(lambda: self.result is not None and predicate(*self.result)),
                               timeout)
        return self.result  # type: ignore[return-value]
    finally:
      self._waiters -= 1

  def on_next(self, fn: Callable[..., Any]) -> None:
    self.observers.append(fn)

  def set(self, *args: T) -> None:
    self.result = args
    for fn in list(self.observers):
      out = fn(*args)
      if asyncio.iscoroutine(out):  # async observers are scheduled on the running loop
        asyncio.get_running_loop().create_task(out)
    if not self._waiters:
      return  # nobody in wait(): no notify task (set() runs once per generated token)
    try:
      asyncio.get_running_loop().create_task(self._notify())
    except RuntimeError:
      pass  # no loop running (sync caller): observers already ran

  async def _notify(self) -> None:
    async with self._cond:
      self._cond.notify_all()


class AsyncCallbackSystem(Generic[K, T]):
  """Named AsyncCallbacks; `trigger_all` fans an event out to every registered name."""

  def __init__(self) -> None:
    self.callbacks: Dict[K, AsyncCallback[T]] = {}

  def register(self, name: K) -> AsyncCallback[T]:
    if name not in self.callbacks:
      self.callbacks[name] = AsyncCallback[T]()
    return self.callbacks[name]

  def deregister(self, name: K) -> None:
    self.callbacks.pop(name, None)

  def trigger(self, name: K, *args: T) -> None:
    if name in self.callbacks:
      self.callbacks[name].set(*args)

  def trigger_all(self, *args: T) -> None:
    for cb in list(self.callbacks.values()):
      cb.set(*args)


# ------------------------------------------------------------------ ports / ids
def _used_ports_file() -> Path:
  return Path(tempfile.gettempdir()) / "xot_used_ports"


def find_available_port(host: str = "", min_port: int = 49152, max_port: int = 65535) -> int:
  """Random free TCP port, avoiding the last 20 handed out on this host."""
  f = _used_ports_file()
  try:
    recent = [int(x) for x in f.read_text().split() if x.isdigit()]
  except OSError:
    recent = []
  avoid = set(recent)
  for _ in range(2000):
    port = random.randint(min_port, max_port)
    if port in avoid:
      continue
    try:
      with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind((host, port))
    except OSError:
      avoid.add(port)
      continue
    try:
      f.write_text("\n".join(str(p) for p in (recent + [port])[-20:]) + "\n")
    except OSError:
      pass
    return port
  raise RuntimeError("No available ports in the specified range")


def get_or_create_node_id() -> str:
  path = Path(tempfile.gettempdir()) / ".xot_node_id"
  try:
    if path.exists():
      nid = path.read_text().strip()
      if nid:
        return nid
    nid = str(uuid.uuid4())
    path.write_text(nid)
    return nid
  except OSError:
    return str(uuid.uuid4())


# ------------------------------------------------------------------ interfaces
# priority: higher is preferred (same ordering as the reference: container > loopback > thunderbolt >
# ethernet > wifi > other > vpn)
_IFACE_RULES = [
  (("docker", "br-", "veth", "cni", "flannel", "calico", "weave"), 7, "Container Virtual"),
  (("lo",), 6, "Loopback"),
  (("tb", "nx", "ten"), 5, "Thunderbolt"),
  (("eth", "en"), 4, "Ethernet"),
  (("wl", "wifi", "wlan"), 3, "WiFi"),
  (("tun", "tap", "vtun", "utun", "gif", "stf", "awdl", "llw", "wg", "tailscale"), 1, "External Virtual"),
]


def get_interface_priority_and_type(ifname: str) -> Tuple[int, str]:
  name = ifname.lower()
  if name == "lo" or name.startswith("lo:"):
    return 6, "Loopback"
  for prefixes, prio, kind in _IFACE_RULES:
    if kind == "Loopback":
      continue
    if name.startswith(prefixes):
      return prio, kind
  return 2, "Other"


def get_all_ip_addresses_and_interfaces() -> List[Tuple[str, str]]:
  out: List[Tuple[str, str]] = []
  try:
    for ifname, addrs in psutil.net_if_addrs().items():
      for a in addrs:
        if a.family == socket.AF_INET and a.address:
          out.append((a.address, ifname))
  except Exception:
    pass
  return out or [("127.0.0.1", "lo")]


def get_broadcast_address(ip: str) -> str:
  try:
    for ifname, addrs in psutil.net_if_addrs().items():
      for a in addrs:
        if a.family == socket.AF_INET and a.address == ip and a.broadcast:
          return a.broadcast
  except Exception:
    pass
  parts = ip.split(".")
  return ".".join(parts[:3] + ["255"]) if len(parts) == 4 else "255.255.255.255"


def xot_home() -> Path:
  return Path(os.environ.get("XOT_HOME", Path.home() / ".cache" / "xot"))


def get_xot_images_dir() -> Path:
  d = xot_home() / "images"
  d.mkdir(parents=True, exist_ok=True)
  return d


async def shutdown(sig: signal.Signals, loop: asyncio.AbstractEventLoop, server=None) -> None:
  """Cancel every task and stop the server (SIGINT/SIGTERM handler)."""
  print(f"Received exit signal {sig.name}...")
  tasks = [t for t in asyncio.all_tasks(loop) if t is not asyncio.current_task()]
  for t in tasks:
    t.cancel()
  await asyncio.gather(*tasks, return_exceptions=True)
  if server is not None:
    await server.stop()
  loop.stop()

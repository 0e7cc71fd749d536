"""Failure detection for the GPU ring: per-rank heartbeats, communicator abort, fault injection.

The reference only has peer liveness at the discovery layer (UDP last-seen + gRPC HealthCheck, peers
dropped after 30 s: xotorch/networking/udp/udp_discovery.py:204-246; manual discovery re-checks every
5 s: manual_discovery.py:52-66) and leaves in-flight requests hanging (node.py:424-443).  The RCCL data
plane needs its own detector: a rank blocked in a recv from a dead neighbour never returns, and RCCL
kernels waiting on a dead peer spin until the process-group timeout (30 min here).

  HealthMonitor   one daemon thread per rank: bumps `xot/hb/<rank>` in the c10d store every
                  `interval` s and watches every other rank's counter; a counter that stops moving for
                  `timeout` s (or a store that stops answering: rank 0 hosts it) marks the rank dead,
                  aborts this rank's communicators (so RCCL kernels and host waits return with an error
                  instead of spinning) and runs the registered callbacks.  A clean `stop()` writes
                  `xot/bye/<rank>` so peers never flag an orderly exit.
  wait_work       host wait on a p2p work handle that polls the monitor, so a rank blocked on a dead
                  neighbour raises PeerFailure (gloo waits block the host; RCCL waits do not).
  FaultInjector   test-only: XOT_FAULT="kill:rank=1:after=3" (rank 1 exits hard on its 4th send),
                  "hang:rank=1:after=3" (stops sending and heartbeating: a wedged peer),
                  "delay:ms=20" (every send sleeps first: a slow link).
After a PeerFailure the survivors re-form the ring with `reform_ring` (a fresh rendezvous of the live
ranks at a new store port) and the caller re-partitions layers over them (ring memory-weighted
partitioner) and re-admits its requests; the Node layer does the same for gRPC peers (_fail_request).
"""
from __future__ import annotations

import datetime
import os
import threading
import time
from typing import Callable, Iterable, List, Optional

import torch.distributed as dist


class PeerFailure(RuntimeError):
  def __init__(self, dead: Iterable[int], why: str = ""):
    self.dead = sorted(set(dead))
    super().__init__(f"ring peer(s) {self.dead} failed" + (f": {why}" if why else ""))


def abort_communicators() -> None:
  """Abort every process group of this rank (RCCL: ncclCommAbort, so kernels spinning on a dead peer
  exit; gloo: pending ops fail).  Safe to call more than once."""
  if not dist.is_initialized():
    return
  try:
    dist.distributed_c10d._abort_process_group()
  except Exception:  # older builds / backends without abort: fall back to a destroy
    try:
      dist.destroy_process_group()
    except Exception:
      pass


def store_port(generation: int = 0) -> int:
  """TCPStore port of ring generation `generation` (0 = the launch rendezvous, n = the n-th re-formed ring)."""
  base = int(os.environ.get("MASTER_PORT", "29500"))
  return base if generation == 0 else base + 1 + generation


def _own_store_client(timeout_s: float = 10.0, generation: int = 0):
  host = os.environ.get("MASTER_ADDR", "127.0.0.1")
  return dist.TCPStore(host, store_port(generation), is_master=False, wait_for_workers=False,
                       timeout=datetime.timedelta(seconds=timeout_s))


class HealthMonitor:
  def __init__(self, rank: int, world: int, store=None, interval: float = 0.25, timeout: float = 3.0,
               abort_on_failure: bool = True, prefix: str = "xot", generation: int = 0):
    self.rank, self.world = rank, world
    # a connection of its own: a TCPStore client is not safe to share with the main thread's
    # rendezvous / new_group traffic
    self.store = store if store is not None else _own_store_client(generation=generation)
    self.interval, self.timeout = interval, timeout
    self.abort_on_failure = abort_on_failure
    self.prefix = prefix
    self.dead: set = set()
    self.why = ""
    self.failed = threading.Event()
    self._stop = threading.Event()
    self._paused = threading.Event()
    self._callbacks: List[Callable[[List[int]], None]] = []
    self._seen = {}  # rank -> (last counter, monotonic time it last changed)
    self._thread: Optional[threading.Thread] = None
    self._beat = 0

  def _key(self, kind: str, r: int) -> str:
    return f"{self.prefix}/{kind}/{r}"

  def on_failure(self, cb: Callable[[List[int]], None]) -> None:
    self._callbacks.append(cb)

  def start(self) -> "HealthMonitor":
    self.store.set(self._key("hb", self.rank), "0")
    now = time.monotonic()
    self._seen = {r: (None, now) for r in range(self.world) if r != self.rank}
    self._thread = threading.Thread(target=self._run, name=f"xot-health-{self.rank}", daemon=True)
    self._thread.start()
    return self

  def stop(self) -> None:
    if self._thread is None:
      return
    try:
      self.store.set(self._key("bye", self.rank), "1")
    except Exception:
      pass
    self._stop.set()
    self._thread.join(timeout=2 * self.interval + 1)
    self._thread = None

  def pause(self) -> None:
    """Stop heartbeating without leaving (fault injection: a wedged peer)."""
    self._paused.set()

  def check(self) -> None:
    if self.failed.is_set():
      raise PeerFailure(self.dead, self.why)

  def alive(self) -> List[int]:
    return [r for r in range(self.world) if r not in self.dead]

  def _declare(self, dead: List[int], why: str) -> None:
    if not dead or self.failed.is_set():
      return
    self.dead.update(dead)
    self.why = why
    self.failed.set()
    if self.abort_on_failure:
      abort_communicators()
    for cb in self._callbacks:
      try:
        cb(sorted(self.dead))
      except Exception:
        pass

  def _run(self) -> None:
    while not self._stop.wait(self.interval):
      try:
        if not self._paused.is_set():
          self._beat += 1
          self.store.set(self._key("hb", self.rank), str(self._beat))
        now = time.monotonic()
        late = []
        for r, (last, t) in self._seen.items():
          if r in self.dead:
            continue
          if self.store.check([self._key("bye", r)]):
            continue  # left cleanly
          v = self.store.get(self._key("hb", r)) if self.store.check([self._key("hb", r)]) else None
          if v != last:
            self._seen[r] = (v, now)
          elif now - t > self.timeout:
            late.append(r)
        if late:
          self._declare(late, f"no heartbeat for {self.timeout:.1f}s")
      except Exception as e:  # the store is hosted by rank 0: losing it means rank 0 is gone
        if self.rank != 0:
          self._declare([0], f"store unreachable ({type(e).__name__})")
        return


def wait_work(work, monitor: Optional[HealthMonitor]) -> None:
  """Host wait on a p2p work handle.  With a monitor the blocking wait runs on a helper thread and this
  thread waits for whichever comes first: the transfer, or the monitor declaring a peer dead (then
  PeerFailure; a gloo wait on a wedged peer is not interrupted by an abort, so the helper is left
  behind, parked on the dead transfer).  A backend error from a closed peer also becomes PeerFailure."""
  if monitor is None:
    work.wait()
    return
  monitor.check()
  done = threading.Event()
  err: list = []

  def _wait():
    try:
      work.wait()
    except Exception as e:  # peer closed the connection / group aborted
      err.append(e)
    done.set()

  threading.Thread(target=_wait, daemon=True).start()
  while not done.wait(monitor.interval):
    monitor.check()
  if err:
    if monitor.failed.wait(timeout=monitor.timeout + 4 * monitor.interval):
      raise PeerFailure(monitor.dead, monitor.why) from err[0]
    raise err[0]


class FaultInjector:
  """Test-only fault injection on the transport (see the module docstring for XOT_FAULT's grammar)."""

  def __init__(self, spec: str, rank: int, monitor: Optional[HealthMonitor] = None):
    self.kind, self.args = "", {}
    if spec:
      parts = spec.split(":")
      self.kind = parts[0]
      for p in parts[1:]:
        k, _, v = p.partition("=")
        self.args[k] = float(v) if "." in v else int(v)
    self.rank, self.monitor = rank, monitor
    self.sends = 0

  @classmethod
  def from_env(cls, rank: int, monitor: Optional[HealthMonitor] = None) -> Optional["FaultInjector"]:
    spec = os.environ.get("XOT_FAULT", "")
    return cls(spec, rank, monitor) if spec else None

  def _mine(self) -> bool:
    return int(self.args.get("rank", self.rank)) == self.rank

  def before_send(self) -> None:
    self.sends += 1
    if not self._mine():
      return
    if self.kind == "delay":
      time.sleep(float(self.args.get("ms", 10)) / 1000.0)
    elif self.sends > int(self.args.get("after", 0)):
      if self.kind == "kill":
        os._exit(17)
      if self.kind == "hang":
        if self.monitor is not None:
          self.monitor.pause()
        while True:
          time.sleep(3600)


def reform_ring(alive: List[int], rank: int, generation: int, backend: Optional[str] = None,
                timeout_s: int = 60) -> tuple:
  """Re-rendezvous the surviving ranks as a new, dense world (new rank = index in `alive`) on a
  fresh TCPStore at store_port(generation) = MASTER_PORT + 1 + generation (generation >= 1).  The old default group must already be aborted.
  Returns (new_rank, new_world)."""
  if rank not in alive:
    raise ValueError(f"rank {rank} is not among the survivors {alive}")
  be = backend or (dist.get_backend() if dist.is_initialized() else "gloo")
  try:
    dist.destroy_process_group()
  except Exception:
    pass
  new_rank, new_world = alive.index(rank), len(alive)
  host = os.environ.get("MASTER_ADDR", "127.0.0.1")
  port = store_port(generation)
  store = dist.TCPStore(host, port, new_world, is_master=new_rank == 0,
                        timeout=datetime.timedelta(seconds=timeout_s))
  dist.init_process_group(be, store=store, rank=new_rank, world_size=new_world,
                          timeout=datetime.timedelta(seconds=timeout_s))
  return new_rank, new_world

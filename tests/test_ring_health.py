"""Failure detection on the ring data plane (parallel/health.py), gloo on CPU, real processes:
a peer that dies (XOT_FAULT=kill) or wedges (XOT_FAULT=hang) mid-stream makes its neighbour raise
PeerFailure within the heartbeat timeout instead of blocking in recv; an orderly exit is not flagged;
the survivors re-form a dense ring and keep communicating.  (The reference's RPC hop just hangs or
logs, xotorch/orchestration/node.py:424-443; SURVEY.md §5 "failure detection".)"""
import os
import socket
import time

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from xotorch_support_jetson_amd.parallel.comm import P2PTransport
from xotorch_support_jetson_amd.parallel.health import FaultInjector, HealthMonitor, PeerFailure, reform_ring

TIMEOUT = 1.5


def _free_port():
  with socket.socket() as s:
    s.bind(("127.0.0.1", 0))
    return s.getsockname()[1]


def _ping_pong(rank, world, port, q, fault, iters):
  os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
  dist.init_process_group("gloo", rank=rank, world_size=world)
  mon = HealthMonitor(rank, world, interval=0.1, timeout=TIMEOUT).start()
  t = P2PTransport(rank, world, monitor=mon, injector=FaultInjector(fault, rank, mon))
  nxt, prv = (rank + 1) % world, (rank - 1) % world
  x = torch.zeros(4)
  t0 = time.monotonic()
  try:
    for i in range(iters):
      if rank == 0:
        t.isend(x + i, nxt)
        t.recv(x, prv)
      else:
        t.recv(x, prv)
        t.isend(x + 1, nxt)
    t.drain()
    mon.stop()
    q.put((rank, "ok", float(x[0]), time.monotonic() - t0))
  except PeerFailure as e:
    q.put((rank, "failure", e.dead, time.monotonic() - t0))
    if fault.startswith("kill") and world == 3:
      # survivors re-form a dense ring and keep going
      alive = [r for r in range(world) if r not in e.dead]
      nr, nw = reform_ring(alive, rank, generation=1, backend="gloo")
      y = torch.tensor([float(rank)])
      dist.all_reduce(y)
      q.put((rank, "reformed", (nr, nw), float(y[0])))
      dist.destroy_process_group()
  q.close()
  q.join_thread()  # flush the queue's feeder thread before the hard exit
  os._exit(0)  # skip interpreter teardown of an aborted group


def _launch(world, fault, iters, wait_s, need):
  port = _free_port()
  ctx = mp.get_context("spawn")
  q = ctx.Queue()
  ps = [ctx.Process(target=_ping_pong, args=(r, world, port, q, fault, iters)) for r in range(world)]
  for p in ps:
    p.start()
  out = []
  deadline = time.monotonic() + wait_s
  try:
    while time.monotonic() < deadline and len(out) < need:
      try:
        out.append(q.get(timeout=0.5))
      except Exception:
        if all(not p.is_alive() for p in ps):
          break
    return out, ps
  finally:
    for p in ps:
      p.join(timeout=1)
      if p.is_alive():
        p.kill()
        p.join()


def test_clean_run_not_flagged():
  out, ps = _launch(2, "", 20, 60, 2)
  res = {r: (s, v) for r, s, v, _ in out}
  assert res[0][0] == "ok" and res[1][0] == "ok", out
  assert res[0][1] == sum(i + 1 for i in range(20))  # rank 0 adds i, rank 1 adds one per trip


def test_killed_peer_raises_peer_failure():
  out, ps = _launch(2, "kill:rank=1:after=3", 50, 60, 1)
  fails = [o for o in out if o[1] == "failure"]
  assert fails and fails[0][0] == 0 and fails[0][2] == [1], out
  assert fails[0][3] < 30  # detected, not the 30-minute process-group timeout
  assert ps[1].exitcode == 17


def test_wedged_peer_detected_by_heartbeat():
  out, ps = _launch(2, "hang:rank=1:after=3", 50, 60, 1)
  fails = [o for o in out if o[1] == "failure"]
  assert fails and fails[0][0] == 0 and fails[0][2] == [1], out
  assert fails[0][3] < TIMEOUT + 20


def test_survivors_reform_ring():
  out, ps = _launch(3, "kill:rank=2:after=2", 50, 90, 4)
  reformed = {o[0]: o for o in out if o[1] == "reformed"}
  assert set(reformed) == {0, 1}, out
  assert reformed[0][2] == (0, 2) and reformed[1][2] == (1, 2)
  assert reformed[0][3] == 1.0  # all-reduce over the new 2-rank world: 0 + 1

"""Discovery (UDP with crossed ports, manual with live reload), event bus, tracing, TUI render
(reference: networking/udp/test_udp_discovery.py, networking/manual/test_manual_discovery.py,
xotorch/test_callbacks.py, viz/test_topology_viz.py)."""
import asyncio
import json
import socket

import pytest

from xotorch_support_jetson_amd.helpers import AsyncCallbackSystem
from xotorch_support_jetson_amd.networking.grpc.grpc_peer_handle import GRPCPeerHandle
from xotorch_support_jetson_amd.networking.grpc.grpc_server import GRPCServer
from xotorch_support_jetson_amd.networking.manual.manual_discovery import ManualDiscovery
from xotorch_support_jetson_amd.networking.udp.udp_discovery import UDPDiscovery
from xotorch_support_jetson_amd.topology.device_capabilities import DeviceCapabilities, DeviceFlops

CAPS = DeviceCapabilities(model="t", chip="t", memory=1000, flops=DeviceFlops(fp32=0, fp16=0, int8=0))


def port(kind=socket.SOCK_STREAM):
  with socket.socket(socket.AF_INET, kind) as s:
    s.bind(("127.0.0.1", 0))
    return s.getsockname()[1]


class _FakeNode:
  """Just enough of a Node for GRPCServer.HealthCheck / CollectTopology."""
  id = "fake"


def handle(pid, addr, desc, caps):
  return GRPCPeerHandle(pid, addr, desc, caps)


def test_manual_discovery_live_reload(tmp_path):
  async def main():
    p1, p2 = port(), port()
    s1, s2 = GRPCServer(_FakeNode(), "127.0.0.1", p1), GRPCServer(_FakeNode(), "127.0.0.1", p2)
    await s1.start()
    await s2.start()
    cfg = tmp_path / "t.json"
    entry = lambda p: {"address": "127.0.0.1", "port": p, "device_capabilities": CAPS.to_dict()}  # noqa: E731
    cfg.write_text(json.dumps({"peers": {"me": entry(p1)}}))
    d = ManualDiscovery(str(cfg), "me", create_peer_handle=handle, poll_interval=0.1)
    await d.start()
    try:
      await asyncio.sleep(0.3)
      assert await d.discover_peers() == []  # only self in the file
      cfg.write_text(json.dumps({"peers": {"me": entry(p1), "other": entry(p2)}}))
      peers = await asyncio.wait_for(d.discover_peers(wait_for_peers=1), 5)
      assert [p.id() for p in peers] == ["other"]
      # peer dies -> dropped after the next health check
      await s2.stop()
      for _ in range(50):
        await asyncio.sleep(0.1)
        if not await d.discover_peers():
          break
      assert await d.discover_peers() == []
    finally:
      await d.stop()
      await s1.stop()

  asyncio.run(asyncio.wait_for(main(), 30))


def test_udp_discovery_crossed_ports():
  async def main():
    ga, gb = port(), port()
    ua, ub = port(socket.SOCK_DGRAM), port(socket.SOCK_DGRAM)
    sa, sb = GRPCServer(_FakeNode(), "0.0.0.0", ga), GRPCServer(_FakeNode(), "0.0.0.0", gb)
    await sa.start()
    await sb.start()
    da = UDPDiscovery("node-a", ga, ua, ub, handle, broadcast_interval=0.2, device_capabilities_override=CAPS)
    db = UDPDiscovery("node-b", gb, ub, ua, handle, broadcast_interval=0.2, device_capabilities_override=CAPS)
    await da.start()
    await db.start()
    try:
      pa = await asyncio.wait_for(da.discover_peers(wait_for_peers=1), 10)
      pb = await asyncio.wait_for(db.discover_peers(wait_for_peers=1), 10)
      assert [p.id() for p in pa] == ["node-b"] and [p.id() for p in pb] == ["node-a"]
      assert await pa[0].health_check()
    finally:
      await da.stop()
      await db.stop()
      await sa.stop()
      await sb.stop()

  try:
    asyncio.run(asyncio.wait_for(main(), 30))
  except asyncio.TimeoutError:
    pytest.skip("no broadcast-capable interface in this sandbox")


def test_async_callback_wait():
  async def main():
    cbs = AsyncCallbackSystem()
    cb = cbs.register("x")
    seen = []
    cb.on_next(lambda *a: seen.append(a))

    async def later():
      await asyncio.sleep(0.05)
      cbs.trigger_all("r", 1, False)
      await asyncio.sleep(0.05)
      cbs.trigger("x", "r", 2, True)

    asyncio.create_task(later())
    res = await cb.wait(lambda rid, n, fin: fin, timeout=2)
    assert res == ("r", 2, True) and len(seen) == 2
    with pytest.raises(asyncio.TimeoutError):
      await cb.wait(lambda rid, n, fin: n == 99, timeout=0.1)

  asyncio.run(main())


def test_tracing_spans_and_traceparent():
  from xotorch_support_jetson_amd.orchestration.tracing import Tracer
  t = Tracer()
  ctx = t.extract("req", {"traceparent": "00-" + "ab" * 16 + "-" + "cd" * 8 + "-01"})
  assert ctx.trace_id == "ab" * 16
  with t.span("process_prompt", request_id="req", node="n0"):
    pass
  for _ in range(25):
    t.on_token("req")
  t.finish("req")
  spans = t.export()
  names = [s["name"] for s in spans]
  assert "process_prompt" in names
  assert sum(1 for n in names if n.startswith("token_group")) >= 2
  assert all(s["trace_id"] == "ab" * 16 for s in spans)
  hdr = t.inject("req2")
  assert hdr["traceparent"].startswith("00-")


def test_topology_viz_renders():
  rich = pytest.importorskip("rich")
  from rich.console import Console

  from xotorch_support_jetson_amd.topology.partitioning_strategy import Partition
  from xotorch_support_jetson_amd.topology.topology import Topology
  from xotorch_support_jetson_amd.viz.topology_viz import TopologyViz
  v = TopologyViz(["http://localhost:52415/v1/chat/completions"], ["http://localhost:52415"], start=False)
  topo = Topology()
  for i in range(4):
    topo.update_node(f"gpu{i}", DeviceCapabilities(model="MI355X", chip="AMD Instinct MI355X", memory=294912,
                                                   flops=DeviceFlops(fp32=157.3, fp16=2516.6, int8=5033.2)))
  topo.active_node_id = "gpu1"
  parts = [Partition(f"gpu{i}", i / 4, (i + 1) / 4) for i in range(4)]
  v.update_visualization(topo, parts, "gpu0", {"gpu2": {"repo_id": "unsloth/llama-3-70b", "status": "in_progress",
                                                        "downloaded_bytes": 50, "total_bytes": 100}})
  v.update_prompt("r", "hello")
  v.update_prompt_output("r", " world")
  c = Console(record=True, width=140)
  c.print(v.render())
  out = c.export_text()
  assert "gpu1" in out and "hello" in out and "50.0%" in out and "GPU rich" in out
  assert "4 Node Cluster" in out and "[0.25-0.50]" in out and "2516.6 TFLOPS" in out


def test_topology_viz_links_layers_and_own_download():
  """The ring panel shows each edge's link description both ways and each peer's layer range; the download
  panel details this node's repo (files, bytes, per-file bars) and summarises the other nodes."""
  pytest.importorskip("rich")
  from datetime import timedelta

  from rich.console import Console

  from xotorch_support_jetson_amd.download.download_progress import RepoFileProgressEvent, RepoProgressEvent
  from xotorch_support_jetson_amd.inference.shard import Shard
  from xotorch_support_jetson_amd.topology.partitioning_strategy import Partition
  from xotorch_support_jetson_amd.topology.topology import Topology
  from xotorch_support_jetson_amd.viz.topology_viz import TopologyViz
  v = TopologyViz(start=False)
  topo = Topology()
  for i in range(3):
    topo.update_node(f"n{i}", DeviceCapabilities(model="MI355X", chip="AMD Instinct MI355X", memory=294912,
                                                 flops=DeviceFlops(fp32=157.3, fp16=2516.6, int8=5033.2)))
  topo.add_edge("n0", "n1", "xGMI")
  topo.add_edge("n1", "n0", "RCCL")
  parts = [Partition("n0", 0.0, 0.5), Partition("n1", 0.5, 0.75), Partition("n2", 0.75, 1.0)]
  f = RepoFileProgressEvent("org/m", "main", "model-00001.safetensors", 30, 30, 120, 10.0, timedelta(seconds=9),
                            "in_progress", 0.0)
  ev = RepoProgressEvent(Shard("m", 0, 39, 80), "org/m", "main", 1, 3, 300, 300, 1200, 2048.0, timedelta(seconds=65),
                         {"model-00001.safetensors": f}, "in_progress")
  v.update_visualization(topo, parts, "n0", {"n0": ev, "n1": ev.to_dict()}, num_layers=80)
  c = Console(record=True, width=140)
  c.print(v.render())
  out = c.export_text()
  assert "xGMI/RCCL" in out and "layers 0-39" in out and "layers 60-79" in out
  assert "(1/3 files)" in out and "model-00001.safetensors" in out and "25%" in out and "ETA 0:01:05" in out
  assert "Other nodes:" in out and "[0.50-0.75]" in out

"""Topology, partitioning and device-capability tests (reference:
xotorch/topology/test_map_partitions.py, test_ring_memory_weighted_partitioning_strategy.py,
test_device_capabilities.py)."""
import json

import pytest

from xotorch_support_jetson_amd.inference.shard import Shard
from xotorch_support_jetson_amd.topology.device_capabilities import (CHIP_FLOPS, UNKNOWN_DEVICE_CAPABILITIES,
                                                                     DeviceCapabilities, DeviceFlops,
                                                                     device_capabilities)
from xotorch_support_jetson_amd.topology.partitioning_strategy import Partition, map_partitions_to_shards
from xotorch_support_jetson_amd.topology.ring_memory_weighted_partitioning_strategy import (
  RingMemoryWeightedPartitioningStrategy, equal_layer_shards)
from xotorch_support_jetson_amd.topology.topology import Topology


def caps(mem, name="x"):
  return DeviceCapabilities(model=name, chip=name, memory=mem, flops=DeviceFlops(fp32=0, fp16=0, int8=0))


def test_map_partitions_rounding():
  parts = [Partition("a", 0.0, 0.42857), Partition("b", 0.42857, 0.71428), Partition("c", 0.71428, 0.99999)]
  assert map_partitions_to_shards(parts, 32, "m") == [Shard("m", 0, 12, 32), Shard("m", 13, 21, 32),
                                                      Shard("m", 22, 31, 32)]
  parts = [Partition("a", 0.0, 0.1), Partition("b", 0.1, 0.2), Partition("c", 0.2, 1.0)]
  assert map_partitions_to_shards(parts, 32, "m") == [Shard("m", 0, 2, 32), Shard("m", 3, 5, 32),
                                                      Shard("m", 6, 31, 32)]
  assert map_partitions_to_shards([Partition("a", 0.0, 1.0)], 32, "m") == [Shard("m", 0, 31, 32)]
  assert map_partitions_to_shards([], 32, "m") == []


def test_map_partitions_tiny_fraction_dropped_and_covering():
  parts = [Partition("a", 0.0, 0.99), Partition("b", 0.99, 1.0)]
  shards = map_partitions_to_shards(parts, 16, "m")
  # every layer is covered exactly once
  covered = [l for s in shards for l in s.layers()]
  assert covered == list(range(16))


def test_ring_memory_weighted():
  t = Topology()
  t.update_node("node1", caps(3000))
  t.update_node("node2", caps(1000))
  t.update_node("node3", caps(6000))
  t.add_edge("node1", "node2")
  t.add_edge("node2", "node3")
  parts = RingMemoryWeightedPartitioningStrategy().partition(t)
  assert parts == [Partition("node3", 0.0, 0.6), Partition("node1", 0.6, 0.9), Partition("node2", 0.9, 1.0)]


def test_ring_memory_weighted_rounding_contiguous():
  t = Topology()
  G = 1024 ** 3
  t.update_node("node1", caps(128 * G))
  t.update_node("node2", caps(192 * G))
  t.update_node("node3", caps(128 * G))
  parts = RingMemoryWeightedPartitioningStrategy().partition(t)
  assert [p.node_id for p in parts] == ["node2", "node3", "node1"]
  assert parts[0].start == 0.0 and parts[0].end == 0.42857
  for a, b in zip(parts, parts[1:]):
    assert a.end == b.start  # contiguous
  assert abs(parts[-1].end - 1.0) < 1e-4


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_equal_layer_shards_70b(world):
  shards = equal_layer_shards("llama-3-70b", 80, world)
  assert len(shards) == world
  assert [s.start_layer for s in shards] == [i * 80 // world for i in range(world)]
  assert shards[-1].end_layer == 79


def test_topology_json_roundtrip_and_merge():
  t = Topology()
  t.update_node("a", caps(10, "A"))
  t.update_node("b", caps(20, "B"))
  t.add_edge("a", "b", "MAN")
  t.active_node_id = "a"
  d = json.loads(json.dumps(t.to_json()))
  t2 = Topology.from_json(d)
  assert t2.get_node("b").memory == 20 and t2.active_node_id == "a"
  assert {(c.from_id, c.to_id, c.description) for c in t2.peer_graph["a"]} == {("a", "b", "MAN")}
  # merge only adopts the peer's own entry and its outgoing edges
  other = Topology()
  other.update_node("b", caps(99, "B"))
  other.update_node("a", caps(1, "stale"))
  other.add_edge("b", "a", "back")
  other.add_edge("a", "zzz", "not-b's")
  t.merge("b", other)
  assert t.get_node("b").memory == 99 and t.get_node("a").memory == 10
  assert "b" in t.peer_graph and all(c.to_id != "zzz" for c in t.peer_graph["a"])


def test_device_capabilities_cpu_and_table():
  c = device_capabilities()
  assert isinstance(c, DeviceCapabilities)
  assert c.memory > 0
  d = c.to_dict()
  assert set(d) >= {"model", "chip", "memory", "flops"}
  # MI355X dense (not 2:1 sparse) numbers
  mi = [v for k, v in CHIP_FLOPS.items() if "MI355X" in k][0]
  assert 2000 < mi.fp16 < 2600
  assert UNKNOWN_DEVICE_CAPABILITIES.memory == 0


def test_device_probes_without_torch_gpu(tmp_path):
  """Jetson (device-tree model + unified MemTotal), macOS system_profiler and amd-smi / rocm-smi JSON
  probes, with fake inputs (the reference mocks subprocess the same way, test_device_capabilities.py)."""
  import json
  from xotorch_support_jetson_amd.topology.device_capabilities import (_lookup_flops, amd_smi_capabilities,
                                                                       jetson_capabilities, mac_capabilities)
  model = tmp_path / "model"
  model.write_bytes(b"NVIDIA Jetson AGX Orin 32GB\x00")
  mem = tmp_path / "meminfo"
  mem.write_text("MemTotal:       31011968 kB\nMemFree:        1000 kB\n")
  j = jetson_capabilities(str(model), str(mem))
  assert j.memory == 31011968 // 1024 and j.flops.fp16 == 35.3
  model.write_bytes(b"Raspberry Pi 5\x00")
  assert jetson_capabilities(str(model), str(mem)) is None
  prof = ("Hardware:\n\n    Hardware Overview:\n\n      Model Name: MacBook Pro\n      Model Identifier: Mac15,9\n"
          "      Chip: Apple M3 Max\n      Memory: 128 GB\n")
  m = mac_capabilities(lambda cmd: prof)
  assert (m.model, m.chip, m.memory) == ("MacBook Pro", "Apple M3 Max", 128 * 1024) and m.flops.fp16 == 28.4
  amd = [{"gpu": 0, "asic": {"market_name": "AMD Instinct MI355X"}, "vram": {"size": {"value": 294896, "unit": "MB"}}},
         {"gpu": 1, "asic": {"market_name": "AMD Instinct MI355X"}, "vram": {"size": {"value": 294896, "unit": "MB"}}}]
  caps = amd_smi_capabilities(lambda cmd: json.dumps(amd) if cmd[0] == "amd-smi" else None)
  assert len(caps) == 2 and caps[1].memory == 294896 and caps[0].flops.fp16 > 2000
  rsmi = {"card0": {"Card Series": "AMD Instinct MI300X", "VRAM Total Memory (B)": str(192 << 30)}}
  caps = amd_smi_capabilities(lambda cmd: json.dumps(rsmi) if cmd[0] == "rocm-smi" else None)
  assert caps[0].memory == 192 << 10 and caps[0].flops.fp16 > 1000
  assert _lookup_flops("Apple M1 Max").fp32 == 10.6 and _lookup_flops("Apple M1").fp32 == 2.29

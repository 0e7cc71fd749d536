"""Ring order = peers sorted by (memory, node_id) descending; each peer's slice of [0,1) is its share of
total memory, boundaries rounded to 5 decimals (reference:
xotorch/topology/ring_memory_weighted_partitioning_strategy.py:7-18).  With 8 equal MI355X peers and
an 80-layer model this gives layers 0-9, 10-19, ..., 70-79."""
from __future__ import annotations

from typing import List

from .partitioning_strategy import Partition, PartitioningStrategy
from .topology import Topology


class RingMemoryWeightedPartitioningStrategy(PartitioningStrategy):
  def partition(self, topology: Topology) -> List[Partition]:
    ranked = sorted(topology.all_nodes(), key=lambda kv: (kv[1].memory, kv[0]), reverse=True)
    total = sum(caps.memory for _, caps in ranked)
    parts: List[Partition] = []
    start = 0.0
    for nid, caps in ranked:
      share = caps.memory / total if total > 0 else 1.0 / len(ranked)
      end = round(start + share, 5)
      parts.append(Partition(nid, start, end))
      start = end
    return parts


def equal_layer_shards(model_id: str, num_layers: int, world: int):
  """Shards for `world` identical GPU peers in device order (peer i = ring position i)."""
  from .device_capabilities import DeviceCapabilities, DeviceFlops
  from .partitioning_strategy import map_partitions_to_shards
  t = Topology()
  for i in range(world):
    # zero-padded ids + equal memory: the (memory, id) descending sort reverses the ids, so name them
    # so that the ring order is device order
    t.update_node(f"gpu{world - 1 - i:03d}", DeviceCapabilities(model="peer", chip="peer", memory=1,
                                                                 flops=DeviceFlops(fp32=0, fp16=0, int8=0)))
  parts = RingMemoryWeightedPartitioningStrategy().partition(t)
  return map_partitions_to_shards(parts, num_layers, model_id)


def memory_weighted_layer_shards(model_id: str, num_layers: int, memories):
  """Shards for GPU peers whose ring order is fixed (process ring: rank r sends to rank r + 1): peer i gets
  a slice of [0, 1) proportional to memories[i], boundaries rounded to 5 decimals exactly as the strategy
  above does, but in the given order instead of sorted by memory.  Equal memories give equal_layer_shards."""
  from .partitioning_strategy import Partition, map_partitions_to_shards
  total = float(sum(memories))
  parts, start = [], 0.0
  for i, m in enumerate(memories):
    share = m / total if total > 0 else 1.0 / len(memories)
    end = round(start + share, 5)
    parts.append(Partition(f"rank{i}", start, end))
    start = end
  shards = map_partitions_to_shards(parts, num_layers, model_id)
  if len(shards) != len(memories):
    raise ValueError(f"{num_layers} layers cannot be split over {len(memories)} peers with memories {list(memories)}")
  return shards

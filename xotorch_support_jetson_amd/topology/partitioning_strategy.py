"""Layer partitioning: fractions of [0, 1) per peer -> contiguous inclusive layer ranges
(reference: xotorch/topology/partitioning_strategy.py:11-42, same rounding semantics)."""
from __future__ import annotations

from abc import ABC, abstractmethod
from dataclasses import dataclass
from typing import List

from ..inference.shard import Shard
from .topology import Topology


@dataclass
class Partition:
  node_id: str
  start: float
  end: float


class PartitioningStrategy(ABC):
  @abstractmethod
  def partition(self, topology: Topology) -> List[Partition]:
    ...


def map_partitions_to_shards(partitions: List[Partition], num_layers: int, model_id: str) -> List[Shard]:
  """floor(start*L) .. floor(end*L)-1 per partition; the last one always reaches layer L-1; empty
  ranges are dropped (so a peer with a tiny fraction can end up with no shard)."""
  shards: List[Shard] = []
  last = len(partitions) - 1
  for i, p in enumerate(partitions):
    lo = int(p.start * num_layers)
    hi = num_layers - 1 if i == last else int(p.end * num_layers) - 1
    if lo <= hi:
      shards.append(Shard(model_id, lo, hi, num_layers))
  if shards and shards[-1].end_layer < num_layers - 1:
    s = shards[-1]
    shards[-1] = Shard(model_id, s.start_layer, num_layers - 1, num_layers)
  return shards

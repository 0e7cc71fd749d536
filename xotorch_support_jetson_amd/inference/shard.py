"""A contiguous, inclusive range of decoder layers of one model (reference: xotorch/inference/shard.py:4-39).

`Shard(model_id, 0, 0, n_layers)` is the "model handle" form the API builds before the node maps
it onto its own partition (reference models.py:237-242, node.py:455-460).
"""
from __future__ import annotations

from dataclasses import asdict, dataclass


@dataclass(frozen=True)
class Shard:
  model_id: str
  start_layer: int
  end_layer: int  # inclusive
  n_layers: int

  def is_first_layer(self) -> bool:
    return self.start_layer == 0

  def is_last_layer(self) -> bool:
    return self.end_layer == self.n_layers - 1

  def get_layer_count(self) -> int:
    return self.end_layer - self.start_layer + 1

  def layers(self) -> range:
    return range(self.start_layer, self.end_layer + 1)

  def to_dict(self) -> dict:
    return asdict(self)

  @staticmethod
  def from_dict(data: dict) -> "Shard":
    return Shard(str(data["model_id"]), int(data["start_layer"]), int(data["end_layer"]), int(data["n_layers"]))

  def overlaps(self, other: "Shard") -> bool:
    return shards_overlap(self, other)

  def key(self) -> str:
    """Deterministic identifier (the reference uses salted hash(shard), node.py:238-239)."""
    return f"{self.model_id}:{self.start_layer:03d}-{self.end_layer:03d}-of-{self.n_layers:03d}"


def shards_overlap(a: Shard, b: Shard) -> bool:
  if a.model_id != b.model_id:
    return False
  return max(a.start_layer, b.start_layer) <= min(a.end_layer, b.end_layer)

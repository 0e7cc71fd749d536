"""Peer graph: node id -> DeviceCapabilities plus directed link descriptions
(reference: xotorch/topology/topology.py:5-75; same JSON shape for /v1/topology)."""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, Optional, Set

from .device_capabilities import DeviceCapabilities


@dataclass(frozen=True)
class PeerConnection:
  from_id: str
  to_id: str
  description: Optional[str] = None

  # identity is the (from, to) pair; the description is payload
  def __hash__(self):
    return hash((self.from_id, self.to_id))

  def __eq__(self, other):
    return isinstance(other, PeerConnection) and (self.from_id, self.to_id) == (other.from_id, other.to_id)


class Topology:
  def __init__(self):
    self.nodes: Dict[str, DeviceCapabilities] = {}
    self.peer_graph: Dict[str, Set[PeerConnection]] = {}
    self.active_node_id: Optional[str] = None

  def update_node(self, node_id: str, caps: DeviceCapabilities) -> None:
    self.nodes[node_id] = caps

  def get_node(self, node_id: str) -> Optional[DeviceCapabilities]:
    return self.nodes.get(node_id)

  def all_nodes(self):
    return self.nodes.items()

  def add_edge(self, from_id: str, to_id: str, description: Optional[str] = None) -> None:
    self.peer_graph.setdefault(from_id, set()).add(PeerConnection(from_id, to_id, description))

  def merge(self, peer_node_id: str, other: "Topology") -> None:
    """Adopt only what the peer is authoritative for: its own node entry and its outgoing edges."""
    if peer_node_id in other.nodes:
      self.update_node(peer_node_id, other.nodes[peer_node_id])
    for conn in other.peer_graph.get(peer_node_id, ()):
      self.add_edge(conn.from_id, conn.to_id, conn.description)

  def to_json(self) -> dict:
    return {
      "nodes": {nid: caps.to_dict() for nid, caps in self.nodes.items()},
      "peer_graph": {nid: [{"from_id": c.from_id, "to_id": c.to_id, "description": c.description} for c in conns]
                     for nid, conns in self.peer_graph.items()},
      "active_node_id": self.active_node_id,
    }

  @staticmethod
  def from_json(d: dict) -> "Topology":
    t = Topology()
    for nid, caps in d.get("nodes", {}).items():
      t.update_node(nid, DeviceCapabilities(**caps))
    for nid, conns in d.get("peer_graph", {}).items():
      for c in conns:
        t.add_edge(c["from_id"], c["to_id"], c.get("description"))
    t.active_node_id = d.get("active_node_id")
    return t

  def __str__(self):
    nodes = ", ".join(f"{k}: {v}" for k, v in self.nodes.items())
    edges = ", ".join(f"{k}: {[f'{c.to_id}({c.description})' for c in v]}" for k, v in self.peer_graph.items())
    return f"Topology(Nodes: {{{nodes}}}, Edges: {{{edges}}})"

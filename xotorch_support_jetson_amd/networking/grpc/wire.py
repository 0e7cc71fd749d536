"""Wire format of the NodeService: the reference protobuf schema (node_service.proto, built at import time
by node_service_pb.py -- no protoc here), so peers built from the reference's generated stubs interoperate.

Tensors travel as Tensor{tensor_data, shape, dtype} with raw little-endian bytes; bf16 activations keep
their 2-byte storage with dtype "bfloat16" (the reference upcasts activations to fp32 and ships its whole
mask / token state as JSON on every hop, grpc_peer_handle.py:117-136, 209-230; a reference peer receiving
bf16 must call the dtype by its torch name, which numpy lacks).  An InferenceState dict is split like the
reference's serialize_inference_state: tensors -> tensor_data, lists of tensors -> tensor_list_data, the
rest -> other_data_json.  gzip channel compression (the reference's default) is opt-in: XOT_GRPC_GZIP=1
(bf16 activations barely compress, and a gRPC server accepts compressed requests either way).
"""
from __future__ import annotations

import json
import os
from typing import Any, Optional

import numpy as np

from .node_service_pb import METHODS, SERVICE, M, method_path  # noqa: F401  (re-exported)

GZIP = os.environ.get("XOT_GRPC_GZIP", "0") == "1"

_NP = {"float32": np.float32, "float16": np.float16, "int64": np.int64, "int32": np.int32, "int16": np.int16,
       "int8": np.int8, "uint8": np.uint8, "float64": np.float64, "bool": np.bool_}


def _is_tensor(v) -> bool:
  if isinstance(v, np.ndarray):
    return True
  try:
    import torch
    return isinstance(v, torch.Tensor)
  except ImportError:  # pragma: no cover
    return False


def encode_tensor(t) -> Optional["M.Tensor"]:
  if t is None:
    return None
  try:
    import torch
    if isinstance(t, torch.Tensor):
      t = t.detach().cpu().contiguous()
      if t.dtype == torch.bfloat16:
        return M.Tensor(tensor_data=t.view(torch.int16).numpy().tobytes(), shape=list(t.shape), dtype="bfloat16")
      t = t.numpy()
  except ImportError:  # pragma: no cover
    pass
  a = np.ascontiguousarray(np.asarray(t))
  return M.Tensor(tensor_data=a.tobytes(), shape=list(a.shape), dtype=str(a.dtype))


def decode_tensor(m: Optional["M.Tensor"]):
  if m is None:
    return None
  shape = list(m.shape)
  if m.dtype == "bfloat16":
    import torch
    raw = np.frombuffer(m.tensor_data, dtype=np.int16).copy()
    return torch.from_numpy(raw).view(torch.bfloat16).reshape(shape)
  return np.frombuffer(m.tensor_data, dtype=_NP.get(m.dtype, m.dtype)).reshape(shape).copy()


def opt_tensor(msg, field: str):
  """An `optional Tensor` field, or None when the sender left it out."""
  return decode_tensor(getattr(msg, field)) if msg.HasField(field) else None


def _json_default(o):
  if isinstance(o, np.generic):
    return o.item()
  if isinstance(o, (set, tuple)):
    return list(o)
  raise TypeError(f"not JSON serialisable: {type(o).__name__}")


def encode_state(state: Optional[dict]) -> Optional["M.InferenceState"]:
  if state is None:
    return None
  m = M.InferenceState()
  other = {}
  for k, v in state.items():
    if _is_tensor(v):
      m.tensor_data[k].CopyFrom(encode_tensor(v))
    elif isinstance(v, (list, tuple)) and v and all(_is_tensor(x) for x in v):
      m.tensor_list_data[k].tensors.extend(encode_tensor(x) for x in v)
    else:
      other[k] = v
  m.other_data_json = json.dumps(other, default=_json_default)
  return m


def decode_state(m: Optional["M.InferenceState"]) -> Optional[dict]:
  if m is None:
    return None
  out: dict = json.loads(m.other_data_json) if m.other_data_json else {}
  for k, t in m.tensor_data.items():
    out[k] = decode_tensor(t)
  for k, tl in m.tensor_list_data.items():
    out[k] = [decode_tensor(t) for t in tl.tensors]
  return out


def opt_state(msg) -> Optional[dict]:
  return decode_state(msg.inference_state) if msg.HasField("inference_state") else None


def encode_topology(d: dict) -> "M.Topology":
  """Topology.to_json() -> Topology message (active_node_id has no field in the schema: not sent)."""
  m = M.Topology()
  for nid, caps in d.get("nodes", {}).items():
    c = m.nodes[nid]
    c.model, c.chip, c.memory = caps["model"], caps["chip"], int(caps["memory"])
    f = caps.get("flops") or {}
    c.flops.fp32, c.flops.fp16, c.flops.int8 = float(f.get("fp32", 0)), float(f.get("fp16", 0)), float(f.get("int8", 0))
  for nid, conns in d.get("peer_graph", {}).items():
    pcs = m.peer_graph[nid]
    for c in conns:
      pc = pcs.connections.add(to_id=c["to_id"])
      if c.get("description") is not None:
        pc.description = c["description"]
  return m


def decode_topology(m: "M.Topology") -> dict:
  """Topology message -> the Topology.from_json shape."""
  nodes = {nid: {"model": c.model, "chip": c.chip, "memory": c.memory,
                 "flops": {"fp32": c.flops.fp32, "fp16": c.flops.fp16, "int8": c.flops.int8}}
           for nid, c in m.nodes.items()}
  graph = {nid: [{"from_id": nid, "to_id": c.to_id, "description": c.description if c.HasField("description") else None}
                 for c in pcs.connections] for nid, pcs in m.peer_graph.items()}
  return {"nodes": nodes, "peer_graph": graph}


def shard_msg(shard) -> "M.Shard":
  return M.Shard(model_id=shard.model_id, start_layer=shard.start_layer, end_layer=shard.end_layer,
                 n_layers=shard.n_layers)


def shard_of(m: "M.Shard"):
  from ...inference.shard import Shard
  return Shard(m.model_id, m.start_layer, m.end_layer, m.n_layers)


def encode(rpc: str, msg) -> bytes:  # noqa: ARG001 - symmetric with decode
  return msg.SerializeToString()


def decode(rpc: str, data: bytes, response: bool = False) -> Any:
  req, resp = METHODS[rpc]
  return (resp if response else req).FromString(data)

"""Wire format of the NodeService (schema documented in node_service.proto next to this file).

Messages are msgpack maps carried by gRPC generic unary methods (this image has grpcio but no protoc,
so there are no generated stubs).  Tensors travel as {"dtype", "shape", "data"} with raw little-endian
bytes; bf16 is sent as its 2-byte storage (the reference upcasts activations to fp32 and JSON-encodes
the whole mask/token state on every hop, grpc_peer_handle.py:117-136, 209-230).
"""
from __future__ import annotations

from typing import Any, Optional

import msgpack
import numpy as np

SERVICE = "xot.NodeService"
METHODS = ("SendPrompt", "SendTensor", "SendExample", "CollectTopology", "SendResult", "SendOpaqueStatus",
           "HealthCheck")

_NP = {"float32": np.float32, "float16": np.float16, "int64": np.int64, "int32": np.int32, "int16": np.int16,
       "uint8": np.uint8, "float64": np.float64, "bool": np.bool_}


def encode_tensor(t) -> Optional[dict]:
  if t is None:
    return None
  try:
    import torch
    if isinstance(t, torch.Tensor):
      t = t.detach().cpu().contiguous()
      if t.dtype == torch.bfloat16:
        return {"dtype": "bfloat16", "shape": list(t.shape), "data": t.view(torch.int16).numpy().tobytes()}
      t = t.numpy()
  except ImportError:  # pragma: no cover
    pass
  a = np.ascontiguousarray(np.asarray(t))
  return {"dtype": str(a.dtype), "shape": list(a.shape), "data": a.tobytes()}


def decode_tensor(d: Optional[dict]):
  if d is None:
    return None
  if d["dtype"] == "bfloat16":
    import torch
    raw = np.frombuffer(d["data"], dtype=np.int16).copy()
    return torch.from_numpy(raw).view(torch.bfloat16).reshape(d["shape"])
  return np.frombuffer(d["data"], dtype=_NP.get(d["dtype"], d["dtype"])).reshape(d["shape"]).copy()


def pack(obj: Any) -> bytes:
  return msgpack.packb(obj, use_bin_type=True)


def unpack(b: bytes) -> Any:
  return msgpack.unpackb(b, raw=False, strict_map_key=False)


def method_path(name: str) -> str:
  return f"/{SERVICE}/{name}"

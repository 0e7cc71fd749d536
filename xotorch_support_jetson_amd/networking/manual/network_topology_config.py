"""Static topology file for manual discovery (reference: xotorch/networking/manual/network_topology_config.py).

{"peers": {"<node id>": {"address": "...", "port": 50051,
                         "device_capabilities": {"model", "chip", "memory", "flops": {"fp32", "fp16", "int8"}}}}}
"""
from __future__ import annotations

from typing import Dict

from pydantic import BaseModel, ValidationError

from ...topology.device_capabilities import DeviceCapabilities


class PeerConfig(BaseModel):
  address: str
  port: int
  device_capabilities: DeviceCapabilities


class NetworkTopology(BaseModel):
  peers: Dict[str, PeerConfig]

  @classmethod
  def from_path(cls, path: str) -> "NetworkTopology":
    try:
      with open(path, "r") as f:
        raw = f.read()
    except FileNotFoundError as e:
      raise FileNotFoundError(f"Config file not found at {path}") from e
    try:
      return cls.model_validate_json(raw)
    except ValidationError as e:
      errs = e.errors()
      if errs and errs[0].get("type") == "json_invalid":
        raise ValueError(f"Error validating network topology config from {path}: invalid JSON") from e
      raise ValueError(f"Error validating network topology config from {path}: {e}") from e

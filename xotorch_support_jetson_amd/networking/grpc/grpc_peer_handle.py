"""gRPC client side of a peer (reference: xotorch/networking/grpc/grpc_peer_handle.py:25-230).

Same channel options (256 MB messages, keepalive, tcp_nodelay) and the reference's protobuf messages and
method paths (wire.py / node_service_pb.py); gzip compression is opt-in (XOT_GRPC_GZIP=1: bf16
activations barely compress).  `send_loss` -- an RPC the reference calls but never defines -- does not
exist here; gradients come back in SendExample's reply (Loss.grads).
"""
from __future__ import annotations

import asyncio
from typing import Optional

import grpc

from ...helpers import DEBUG
from ...inference.shard import Shard
from ...topology.device_capabilities import DeviceCapabilities
from ...topology.topology import Topology
from ..peer_handle import PeerHandle
from .wire import (GZIP, METHODS, M, decode_topology, encode_state, encode_tensor, method_path, opt_tensor,
                   shard_msg)

CHANNEL_OPTIONS = [
  ("grpc.max_metadata_size", 32 * 1024 * 1024),
  ("grpc.max_receive_message_length", 256 * 1024 * 1024),
  ("grpc.max_send_message_length", 256 * 1024 * 1024),
  ("grpc.max_concurrent_streams", 100),
  ("grpc.http2.min_time_between_pings_ms", 10000),
  ("grpc.keepalive_time_ms", 10000),
  ("grpc.keepalive_timeout_ms", 5000),
  ("grpc.keepalive_permit_without_calls", 1),
  ("grpc.http2.max_pings_without_data", 0),
  ("grpc.tcp_nodelay", 1),
  ("grpc.optimization_target", "throughput"),
]


class GRPCPeerHandle(PeerHandle):
  def __init__(self, _id: str, address: str, desc: str, device_capabilities: DeviceCapabilities):
    self._id = _id
    self.address = address
    self.desc = desc
    self._caps = device_capabilities
    self.channel: Optional[grpc.aio.Channel] = None
    self._calls = {}

  def id(self) -> str:
    return self._id

  def addr(self) -> str:
    return self.address

  def description(self) -> str:
    return self.desc

  def device_capabilities(self) -> DeviceCapabilities:
    return self._caps

  async def connect(self):
    if self.channel is None:
      self.channel = grpc.aio.insecure_channel(self.address, options=CHANNEL_OPTIONS)
      self._calls = {}
    await asyncio.wait_for(self.channel.channel_ready(), timeout=10.0)

  async def is_connected(self) -> bool:
    return self.channel is not None and self.channel.get_state() == grpc.ChannelConnectivity.READY

  async def disconnect(self):
    if self.channel is not None:
      await self.channel.close()
    self.channel = None
    self._calls = {}

  async def _ensure_connected(self):
    if not await self.is_connected():
      try:
        await asyncio.wait_for(self.connect(), timeout=10.0)
      except asyncio.TimeoutError:
        if DEBUG >= 2:
          print(f"connection timeout to {self._id}@{self.address}")
        raise

  def _call(self, name: str):
    if name not in self._calls:
      req, resp = METHODS[name]
      self._calls[name] = self.channel.unary_unary(method_path(name), request_serializer=req.SerializeToString,
                                                   response_deserializer=resp.FromString)
    return self._calls[name]

  async def _rpc(self, name: str, msg, timeout: Optional[float] = None):
    await self._ensure_connected()
    kw = {"compression": grpc.Compression.Gzip} if GZIP else {}
    return await self._call(name)(msg, timeout=timeout, **kw)

  async def health_check(self, timeout: float = 3.0) -> bool:
    try:
      r = await asyncio.wait_for(self._rpc("HealthCheck", M.HealthCheckRequest(), timeout=timeout), timeout)
      return bool(r is not None and r.is_healthy)
    except asyncio.TimeoutError:
      return False
    except Exception:
      if DEBUG >= 4:
        import traceback
        traceback.print_exc()
      return False

  async def send_prompt(self, shard: Shard, prompt: str, request_id: Optional[str] = None,
                        inference_state: Optional[dict] = None) -> None:
    m = M.PromptRequest(shard=shard_msg(shard), prompt=prompt)
    if request_id is not None:
      m.request_id = request_id
    if inference_state is not None:
      m.inference_state.CopyFrom(encode_state(inference_state))
    await self._rpc("SendPrompt", m)

  async def send_tensor(self, shard: Shard, tensor, request_id: Optional[str] = None,
                        inference_state: Optional[dict] = None) -> None:
    m = M.TensorRequest(shard=shard_msg(shard), tensor=encode_tensor(tensor))
    if request_id is not None:
      m.request_id = request_id
    if inference_state is not None:
      m.inference_state.CopyFrom(encode_state(inference_state))
    await self._rpc("SendTensor", m)

  async def send_example(self, shard: Shard, example, target, length, train: bool,
                         request_id: Optional[str] = None):
    m = M.ExampleRequest(shard=shard_msg(shard), example=encode_tensor(example), target=encode_tensor(target),
                         length=encode_tensor(length), train=bool(train))
    if request_id is not None:
      m.request_id = request_id
    r = await self._rpc("SendExample", m)
    grads = opt_tensor(r, "grads")
    return (float(r.loss), grads) if train else float(r.loss)

  async def send_result(self, request_id: str, result, is_finished: bool) -> None:
    m = M.SendResultRequest(request_id=request_id, is_finished=bool(is_finished))
    if hasattr(result, "shape") and getattr(result, "ndim", 1) > 1:
      m.tensor.CopyFrom(encode_tensor(result))
    else:
      m.result.extend(int(x) for x in result)
    await self._rpc("SendResult", m, timeout=15)

  async def send_opaque_status(self, request_id: str, status: str) -> None:
    await self._rpc("SendOpaqueStatus", M.SendOpaqueStatusRequest(request_id=request_id, status=status), timeout=10)

  async def collect_topology(self, visited: set, max_depth: int) -> Topology:
    r = await self._rpc("CollectTopology", M.CollectTopologyRequest(visited=sorted(visited), max_depth=int(max_depth)),
                        timeout=5)
    return Topology.from_json(decode_topology(r))

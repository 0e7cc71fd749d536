"""gRPC server side of a node (reference: xotorch/networking/grpc/grpc_server.py:21-173).

Generic method handlers dispatch msgpack messages to the Node; every handler is async (grpc.aio), so
the server does not need the reference's 32-thread pool.
"""
from __future__ import annotations

import grpc

from ...helpers import DEBUG
from ...inference.shard import Shard
from ..server import Server
from .grpc_peer_handle import CHANNEL_OPTIONS
from .wire import SERVICE, decode_tensor, encode_tensor, pack, unpack


class GRPCServer(Server):
  def __init__(self, node, host: str, port: int):
    self.node = node
    self.host = host
    self.port = port
    self.server = None

  async def start(self) -> None:
    self.server = grpc.aio.server(options=CHANNEL_OPTIONS)
    handlers = {name: grpc.unary_unary_rpc_method_handler(getattr(self, name), request_deserializer=lambda b: b,
                                                          response_serializer=lambda b: b)
                for name in ("SendPrompt", "SendTensor", "SendExample", "CollectTopology", "SendResult",
                             "SendOpaqueStatus", "HealthCheck")}
    self.server.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(SERVICE, handlers),))
    listen = f"{self.host}:{self.port}"
    self.server.add_insecure_port(listen)
    await self.server.start()
    if DEBUG >= 1:
      print(f"Server started, listening on {listen}")

  async def stop(self) -> None:
    if self.server:
      try:
        await self.server.stop(grace=5)
        await self.server.wait_for_termination()
      except Exception:
        pass
      if DEBUG >= 1:
        print("Server stopped and all connections are closed")

  # ---------------------------------------------------------------- handlers
  async def SendPrompt(self, request: bytes, context) -> bytes:
    m = unpack(request)
    shard = Shard.from_dict(m["shard"])
    await self.node.process_prompt(shard, m["prompt"], m.get("request_id"), m.get("inference_state"))
    return pack({})

  async def SendTensor(self, request: bytes, context) -> bytes:
    m = unpack(request)
    shard = Shard.from_dict(m["shard"])
    tensor = decode_tensor(m["tensor"])
    await self.node.process_tensor(shard, tensor, m.get("request_id"), m.get("inference_state"))
    return pack({})

  async def SendExample(self, request: bytes, context) -> bytes:
    m = unpack(request)
    shard = Shard.from_dict(m["shard"])
    example, target, length = decode_tensor(m["example"]), decode_tensor(m["target"]), decode_tensor(m["length"])
    train = bool(m.get("train"))
    res = await self.node.process_example(shard, example, target, length, train, m.get("request_id"))
    if train:
      loss, grads = res
      return pack({"loss": float(loss), "grads": encode_tensor(grads)})
    return pack({"loss": float(res), "grads": None})

  async def CollectTopology(self, request: bytes, context) -> bytes:
    m = unpack(request)
    topo = await self.node.collect_topology(set(m.get("visited", [])), int(m.get("max_depth", 4)))
    return pack(topo.to_json())

  async def SendResult(self, request: bytes, context) -> bytes:
    m = unpack(request)
    result = m.get("result") or []
    if m.get("tensor") is not None:
      result = decode_tensor(m["tensor"])
    self.node.on_token.trigger_all(m["request_id"], result, bool(m.get("is_finished")))
    return pack({})

  async def SendOpaqueStatus(self, request: bytes, context) -> bytes:
    m = unpack(request)
    self.node.on_opaque_status.trigger_all(m["request_id"], m["status"])
    return pack({})

  async def HealthCheck(self, request: bytes, context) -> bytes:
    return pack({"is_healthy": True})

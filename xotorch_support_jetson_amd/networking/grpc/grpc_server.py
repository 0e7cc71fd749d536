"""gRPC server side of a node (reference: xotorch/networking/grpc/grpc_server.py:21-173).

Serves the reference's NodeService (protobuf messages and method paths: wire.py / node_service_pb.py) with
async handlers (grpc.aio), so it needs no 32-thread pool; requests compressed with gzip are accepted.
"""
from __future__ import annotations

import grpc

from ...helpers import DEBUG
from ..server import Server
from .grpc_peer_handle import CHANNEL_OPTIONS
from .wire import METHODS, SERVICE, M, decode_tensor, encode_tensor, encode_topology, opt_state, shard_of


class GRPCServer(Server):
  def __init__(self, node, host: str, port: int):
    self.node = node
    self.host = host
    self.port = port
    self.server = None

  async def start(self) -> None:
    self.server = grpc.aio.server(options=CHANNEL_OPTIONS)
    handlers = {name: grpc.unary_unary_rpc_method_handler(getattr(self, name), request_deserializer=req.FromString,
                                                          response_serializer=resp.SerializeToString)
                for name, (req, resp) in METHODS.items()}
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
  @staticmethod
  def _rid(m):
    return m.request_id if m.HasField("request_id") else None

  async def SendPrompt(self, m, context):
    await self.node.process_prompt(shard_of(m.shard), m.prompt, self._rid(m), opt_state(m))
    return M.Tensor()

  async def SendTensor(self, m, context):
    await self.node.process_tensor(shard_of(m.shard), decode_tensor(m.tensor), self._rid(m), opt_state(m))
    return M.Tensor()

  async def SendExample(self, m, context):
    example, target, length = decode_tensor(m.example), decode_tensor(m.target), decode_tensor(m.length)
    res = await self.node.process_example(shard_of(m.shard), example, target, length, bool(m.train), self._rid(m))
    if m.train:
      loss, grads = res
      out = M.Loss(loss=float(loss))
      if grads is not None:
        out.grads.CopyFrom(encode_tensor(grads))
      return out
    return M.Loss(loss=float(res))

  async def CollectTopology(self, m, context):
    topo = await self.node.collect_topology(set(m.visited), int(m.max_depth) or 4)
    return encode_topology(topo.to_json())

  async def SendResult(self, m, context):
    result = decode_tensor(m.tensor) if m.HasField("tensor") else list(m.result)
    self.node.on_token.trigger_all(m.request_id, result, bool(m.is_finished))
    return M.Empty()

  async def SendOpaqueStatus(self, m, context):
    self.node.on_opaque_status.trigger_all(m.request_id, m.status)
    return M.Empty()

  async def HealthCheck(self, m, context):
    return M.HealthCheckResponse(is_healthy=True)

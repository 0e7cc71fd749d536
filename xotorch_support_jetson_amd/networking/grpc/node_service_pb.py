"""The NodeService protobuf schema (node_service.proto next to this file), built at import time.

This image has the protobuf runtime but no protoc, so instead of generated `_pb2` modules the file
descriptor is assembled here field by field from descriptor_pb2 and registered in a private pool; the
message classes come from message_factory.  Package, service, message and field names and numbers are
those of the reference schema (xotorch/networking/grpc/node_service.proto:1-116), so the bytes on the wire
and the method paths (/node_service.NodeService/SendTensor, ...) are the reference's: a peer built from
its generated stubs decodes what this one sends and vice versa.

  M.Tensor, M.PromptRequest, ...     message classes
  METHODS                            name -> (request class, response class)
  SERVICE                            "node_service.NodeService"
"""
from __future__ import annotations

from types import SimpleNamespace

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

PACKAGE = "node_service"
SERVICE = f"{PACKAGE}.NodeService"

F = descriptor_pb2.FieldDescriptorProto
_T = {"string": F.TYPE_STRING, "int32": F.TYPE_INT32, "bytes": F.TYPE_BYTES, "bool": F.TYPE_BOOL,
      "float": F.TYPE_FLOAT, "double": F.TYPE_DOUBLE}

# message -> [(field, number, type, label)]; type is a scalar name or a message name; label: "" (singular),
# "opt" (proto3 optional), "rep" (repeated), ("map", key type, value type)
_SCHEMA = {
  "Shard": [("model_id", 1, "string", ""), ("start_layer", 2, "int32", ""), ("end_layer", 3, "int32", ""),
            ("n_layers", 4, "int32", "")],
  "PromptRequest": [("shard", 1, "Shard", ""), ("prompt", 2, "string", ""), ("request_id", 3, "string", "opt"),
                    ("inference_state", 4, "InferenceState", "opt")],
  "TensorRequest": [("shard", 1, "Shard", ""), ("tensor", 2, "Tensor", ""), ("request_id", 3, "string", "opt"),
                    ("inference_state", 4, "InferenceState", "opt")],
  "ExampleRequest": [("shard", 1, "Shard", ""), ("example", 2, "Tensor", ""), ("target", 3, "Tensor", ""),
                     ("length", 4, "Tensor", ""), ("train", 5, "bool", ""), ("request_id", 6, "string", "opt")],
  "Loss": [("loss", 1, "float", ""), ("grads", 2, "Tensor", "opt")],
  "Tensor": [("tensor_data", 1, "bytes", ""), ("shape", 2, "int32", "rep"), ("dtype", 3, "string", "")],
  "TensorList": [("tensors", 1, "Tensor", "rep")],
  "InferenceState": [("tensor_data", 1, "Tensor", ("map", "string")),
                     ("tensor_list_data", 2, "TensorList", ("map", "string")),
                     ("other_data_json", 3, "string", "")],
  "CollectTopologyRequest": [("visited", 1, "string", "rep"), ("max_depth", 2, "int32", "")],
  "Topology": [("nodes", 1, "DeviceCapabilities", ("map", "string")),
               ("peer_graph", 2, "PeerConnections", ("map", "string"))],
  "PeerConnection": [("to_id", 1, "string", ""), ("description", 2, "string", "opt")],
  "PeerConnections": [("connections", 1, "PeerConnection", "rep")],
  "DeviceFlops": [("fp32", 1, "double", ""), ("fp16", 2, "double", ""), ("int8", 3, "double", "")],
  "DeviceCapabilities": [("model", 1, "string", ""), ("chip", 2, "string", ""), ("memory", 3, "int32", ""),
                         ("flops", 4, "DeviceFlops", "")],
  "SendResultRequest": [("request_id", 1, "string", ""), ("result", 2, "int32", "rep"), ("tensor", 3, "Tensor", "opt"),
                        ("is_finished", 4, "bool", "")],
  "SendOpaqueStatusRequest": [("request_id", 1, "string", ""), ("status", 2, "string", "")],
  "HealthCheckRequest": [],
  "HealthCheckResponse": [("is_healthy", 1, "bool", "")],
  "Empty": [],
}

_RPCS = [("SendPrompt", "PromptRequest", "Tensor"), ("SendTensor", "TensorRequest", "Tensor"),
         ("SendExample", "ExampleRequest", "Loss"), ("CollectTopology", "CollectTopologyRequest", "Topology"),
         ("SendResult", "SendResultRequest", "Empty"), ("SendOpaqueStatus", "SendOpaqueStatusRequest", "Empty"),
         ("HealthCheck", "HealthCheckRequest", "HealthCheckResponse")]


def _set_type(f, typ: str) -> None:
  if typ in _T:
    f.type = _T[typ]
  else:
    f.type = F.TYPE_MESSAGE
    f.type_name = f".{PACKAGE}.{typ}"


def _file() -> descriptor_pb2.FileDescriptorProto:
  fdp = descriptor_pb2.FileDescriptorProto(name="node_service.proto", package=PACKAGE, syntax="proto3")
  for name, fields in _SCHEMA.items():
    m = fdp.message_type.add(name=name)
    for fname, num, typ, label in fields:
      f = m.field.add(name=fname, number=num, json_name="".join(
        p if i == 0 else p.capitalize() for i, p in enumerate(fname.split("_"))))
      if isinstance(label, tuple):  # map<key, value>: a repeated nested *Entry message
        entry = "".join(p.capitalize() for p in fname.split("_")) + "Entry"
        e = m.nested_type.add(name=entry)
        e.options.map_entry = True
        k = e.field.add(name="key", number=1, label=F.LABEL_OPTIONAL, json_name="key")
        _set_type(k, label[1])
        v = e.field.add(name="value", number=2, label=F.LABEL_OPTIONAL, json_name="value")
        _set_type(v, typ)
        f.label = F.LABEL_REPEATED
        f.type = F.TYPE_MESSAGE
        f.type_name = f".{PACKAGE}.{name}.{entry}"
        continue
      f.label = F.LABEL_REPEATED if label == "rep" else F.LABEL_OPTIONAL
      _set_type(f, typ)
      if label == "opt":  # proto3 `optional`: a synthetic one-field oneof named _<field>
        f.proto3_optional = True
        f.oneof_index = len(m.oneof_decl)
        m.oneof_decl.add(name=f"_{fname}")
  svc = fdp.service.add(name="NodeService")
  for rpc, req, resp in _RPCS:
    svc.method.add(name=rpc, input_type=f".{PACKAGE}.{req}", output_type=f".{PACKAGE}.{resp}")
  return fdp


_pool = descriptor_pool.DescriptorPool()
FILE = _pool.Add(_file())
M = SimpleNamespace(**{name: message_factory.GetMessageClass(_pool.FindMessageTypeByName(f"{PACKAGE}.{name}"))
                       for name in _SCHEMA})
METHODS = {rpc: (getattr(M, req), getattr(M, resp)) for rpc, req, resp in _RPCS}


def method_path(name: str) -> str:
  return f"/{SERVICE}/{name}"

"""CPU unit tests for the model registry, configs, block managers, wire codec, dataset, tokenizers,
manual-discovery config (reference: test/test_model_helpers.py, test/test_tokenizers.py,
xotorch/networking/manual/test_network_topology_config.py)."""
import json
import os

import numpy as np
import pytest
import torch

from xotorch_support_jetson_amd.inference.shard import Shard
from xotorch_support_jetson_amd.models import registry as R
from xotorch_support_jetson_amd.models.config import PRESETS, from_hf_config


# ---------------------------------------------------------------- registry / config
def test_model_cards_and_shards():
  E = R.ENGINE
  assert R.build_base_shard("llama-3-70b", E) == Shard("llama-3-70b", 0, 0, 80)
  assert R.build_full_shard("llama-3.2-1b", E) == Shard("llama-3.2-1b", 0, 15, 16)
  assert R.build_base_shard("dummy", "DummyInferenceEngine").n_layers == 8
  assert R.build_base_shard("no-such-model", E) is None
  assert R.get_repo("llama-3.2-1b", E) == "unsloth/Llama-3.2-1B-Instruct"
  assert R.get_pretty_name("llama-3.3-70b") == "Llama 3.3 70B"


def test_supported_models_intersection():
  both = R.get_supported_models([["mi355x"], ["mi355x", "dummy"]])
  assert "llama-3-70b" in both and "dummy" not in both
  assert R.get_supported_models([["dummy"]]) == ["dummy"]
  assert len(R.get_supported_models()) == len(R.model_cards)


def test_validate_layers_warns():
  with pytest.warns(UserWarning):
    assert R.validate_layers("llama-3.2-1b", 17) == 17


def test_presets_match_hf_shapes():
  c = PRESETS["llama-3-70b"]
  assert (c.num_layers, c.hidden_size, c.num_heads, c.num_kv_heads, c.intermediate_size, c.vocab_size) == \
         (80, 8192, 64, 8, 28672, 128256)
  for name, cfg in PRESETS.items():
    assert cfg.is_mla or cfg.hidden_size == cfg.num_heads * cfg.head_dim or cfg.head_dim in (64, 128), name
  # every model card with a preset agrees on the layer count; parameter totals of the big dense cards
  for name, card in R.model_cards.items():
    if name in PRESETS:
      assert PRESETS[name].num_layers == card["layers"], name
  for name, billions in (("llama-3.1-405b", 405.9), ("qwen-2.5-72b", 72.7), ("mistral-large", 122.6),
                         ("qwen-2.5-32b", 32.8), ("llama-3-8b", 8.0), ("deepseek-v3", 671.0),
                         ("deepseek-coder-v2-lite", 15.7), ("phi-4-mini-instruct", 3.84), ("llava-1.5-7b-hf", 6.76)):
    assert abs(PRESETS[name].num_params() / 1e9 - billions) < 0.15, name


def test_config_from_hf_dict():
  hf = {"architectures": ["LlamaForCausalLM"], "model_type": "llama", "hidden_size": 2048, "num_hidden_layers": 16,
        "num_attention_heads": 32, "num_key_value_heads": 8, "intermediate_size": 8192, "vocab_size": 128256,
        "rms_norm_eps": 1e-5, "rope_theta": 500000.0, "tie_word_embeddings": True,
        "rope_scaling": {"rope_type": "llama3", "factor": 32.0, "low_freq_factor": 1.0, "high_freq_factor": 4.0,
                         "original_max_position_embeddings": 8192}}
  c = from_hf_config(hf)
  assert c.head_dim == 64 and c.tie_word_embeddings and c.num_layers == 16


# ---------------------------------------------------------------- block managers
def _managers():
  from xotorch_support_jetson_amd.runtime.block_manager_py import BlockManager as PyBM
  out = [PyBM]
  try:
    from xotorch_support_jetson_amd import _runtime
    out.append(_runtime.BlockManager)
  except ImportError:
    pass
  return out


@pytest.mark.parametrize("BM", _managers())
def test_block_manager_semantics(BM):
  bm = BM(8, 64)
  assert bm.num_free == 8
  s = bm.append("a", 100)
  assert len(s) == 100 and bm.num_tokens("a") == 100
  tab = bm.block_table("a")
  assert len(tab) == 2
  assert s[0] == tab[0] * 64 and s[99] == tab[1] * 64 + 35
  assert bm.blocks_needed("a", 28) == 0 and bm.blocks_needed("a", 29) == 1
  bm.append("b", 64)
  assert bm.num_free == 5
  assert not bm.can_append("c", 6 * 64)
  bm.truncate("a", 10)
  assert bm.num_free == 6 and bm.num_tokens("a") == 10
  tables = np.zeros((2, 4), dtype=np.int32)
  ctx = np.zeros(2, dtype=np.int32)
  bm.fill_batch(["a", "b"], tables, ctx)
  assert list(ctx) == [10, 64] and tables[0, 0] == bm.block_table("a")[0]
  bm.free("a")
  bm.append("a", 100)
  bm.fork("a", "a2", 100)  # shares only the full pages: 64 tokens, 1 refcounted page
  assert bm.num_tokens("a2") == 64 and bm.num_free == 5
  bm.free("a")
  assert bm.num_free == 6  # the shared page stays alive for a2
  bm.free("a2")
  bm.free("b")
  assert bm.num_free == 8 and not bm.has("b")


def test_block_manager_native_matches_python():
  mgrs = _managers()
  if len(mgrs) < 2:
    pytest.skip("native runtime not built")
  rng = np.random.default_rng(0)
  a, b = mgrs[0](64, 64), mgrs[1](64, 64)
  live = []
  for step in range(300):
    op = rng.integers(0, 3)
    if op == 0 or not live:
      rid = f"r{step}"
      n = int(rng.integers(1, 200))
      if a.can_append(rid, n):
        assert a.append(rid, n) == b.append(rid, n)
        live.append(rid)
    elif op == 1:
      rid = live[int(rng.integers(0, len(live)))]
      if a.can_append(rid, 1):
        assert a.append(rid, 1) == b.append(rid, 1)
    else:
      rid = live.pop(int(rng.integers(0, len(live))))
      a.free(rid)
      b.free(rid)
    assert a.num_free == b.num_free


# ---------------------------------------------------------------- wire codec
def test_wire_roundtrip():
  from xotorch_support_jetson_amd.networking.grpc import wire
  x = np.arange(12, dtype=np.float32).reshape(3, 4)
  y = wire.decode_tensor(wire.encode_tensor(x))
  assert y.dtype == np.float32 and (y == x).all()
  t = torch.randn(2, 3, 5).to(torch.bfloat16)
  t2 = wire.decode_tensor(wire.M.Tensor.FromString(wire.encode_tensor(t).SerializeToString()))
  assert t2.dtype == torch.bfloat16 and torch.equal(t2, t)
  assert wire.decode_tensor(wire.encode_tensor(None)) is None
  ids = np.array([[1, 2, 3]], dtype=np.int64)
  assert (wire.decode_tensor(wire.encode_tensor(ids)) == ids).all()
  st = {"n_past": 3, "pc": {"save": [0, 192]}, "h": torch.ones(2, 2).to(torch.bfloat16), "l": [np.zeros(3, np.int32)],
        "temperature": np.float32(0.5)}
  back = wire.decode_state(wire.M.InferenceState.FromString(wire.encode_state(st).SerializeToString()))
  assert back["n_past"] == 3 and back["pc"] == {"save": [0, 192]} and back["temperature"] == 0.5
  assert torch.equal(back["h"], st["h"]) and (back["l"][0] == 0).all()


def test_node_service_messages_roundtrip():
  """Every message of the reference schema (xotorch/networking/grpc/node_service.proto:15-116) encodes and
  decodes through the runtime-built descriptors, optional fields keep their presence."""
  from xotorch_support_jetson_amd.networking.grpc.node_service_pb import METHODS, M, SERVICE, method_path
  tens = M.Tensor(tensor_data=b"\x01\x02", shape=[1, 2], dtype="uint8")
  sh = M.Shard(model_id="llama-3-70b", start_layer=10, end_layer=19, n_layers=80)
  st = M.InferenceState(other_data_json='{"n_past": 4}')
  st.tensor_data["x"].CopyFrom(tens)
  st.tensor_list_data["y"].tensors.extend([tens, tens])
  topo = M.Topology()
  topo.nodes["a"].CopyFrom(M.DeviceCapabilities(model="MI355X", chip="gfx950", memory=288 * 1024,
                                                flops=M.DeviceFlops(fp32=157.3, fp16=2500.0, int8=5000.0)))
  topo.peer_graph["a"].connections.add(to_id="b", description="xGMI")
  topo.peer_graph["a"].connections.add(to_id="c")
  msgs = [sh, tens, st, topo, M.TensorList(tensors=[tens]),
          M.PromptRequest(shard=sh, prompt="hi", request_id="r", inference_state=st),
          M.TensorRequest(shard=sh, tensor=tens, request_id="r", inference_state=st),
          M.ExampleRequest(shard=sh, example=tens, target=tens, length=tens, train=True, request_id="r"),
          M.Loss(loss=1.5, grads=tens), M.CollectTopologyRequest(visited=["a", "b"], max_depth=4),
          M.PeerConnection(to_id="b", description="d"), M.PeerConnections(connections=[M.PeerConnection(to_id="z")]),
          M.DeviceFlops(fp32=1.0, fp16=2.0, int8=4.0), M.DeviceCapabilities(model="m", chip="c", memory=1),
          M.SendResultRequest(request_id="r", result=[1, 2, 3], tensor=tens, is_finished=True),
          M.SendOpaqueStatusRequest(request_id="r", status="{}"), M.HealthCheckRequest(),
          M.HealthCheckResponse(is_healthy=True), M.Empty()]
  for m in msgs:
    assert type(m).FromString(m.SerializeToString()) == m, type(m).__name__
  bare = M.TensorRequest.FromString(M.TensorRequest(shard=sh, tensor=tens).SerializeToString())
  assert not bare.HasField("request_id") and not bare.HasField("inference_state")
  assert not M.PeerConnection.FromString(M.PeerConnection(to_id="x").SerializeToString()).HasField("description")
  assert SERVICE == "node_service.NodeService" and method_path("SendTensor") == "/node_service.NodeService/SendTensor"
  assert set(METHODS) == {"SendPrompt", "SendTensor", "SendExample", "CollectTopology", "SendResult",
                          "SendOpaqueStatus", "HealthCheck"}


def test_node_service_descriptor_matches_reference():
  """Wire compatibility: the runtime-built file descriptor equals the one the reference's generated stubs
  register (read from node_service_pb2.py's serialized descriptor with ast -- nothing of it is executed)."""
  import ast
  import pathlib

  from google.protobuf import descriptor_pb2

  from xotorch_support_jetson_amd.networking.grpc.node_service_pb import FILE
  ref = pathlib.Path("/root/reference/xotorch/networking/grpc/node_service_pb2.py")
  if not ref.exists():
    pytest.skip("reference checkout not present")
  blob = None
  for node in ast.walk(ast.parse(ref.read_text())):
    if isinstance(node, ast.Call) and getattr(node.func, "attr", "") == "AddSerializedFile":
      blob = ast.literal_eval(node.args[0])
  assert blob is not None
  theirs = descriptor_pb2.FileDescriptorProto.FromString(blob)
  ours = descriptor_pb2.FileDescriptorProto()
  FILE.CopyToProto(ours)
  assert ours.package == theirs.package and [s.name for s in ours.service] == [s.name for s in theirs.service]
  assert [(m.name, m.input_type, m.output_type) for m in ours.service[0].method] == \
         [(m.name, m.input_type, m.output_type) for m in theirs.service[0].method]

  def fields(fdp):
    out = {}
    for m in fdp.message_type:
      for f in m.field:
        out[(m.name, f.name)] = (f.number, f.type, f.label, f.type_name, f.proto3_optional)
      for n in m.nested_type:
        for f in n.field:
          out[(m.name + "." + n.name, f.name)] = (f.number, f.type, f.label, f.type_name, n.options.map_entry)
    return out
  assert fields(ours) == fields(theirs)


# ---------------------------------------------------------------- dataset
def test_dataset_batches():
  from xotorch_support_jetson_amd.train.dataset import batch_with_lengths, iterate_batches, load_dataset
  x, y, ln = batch_with_lengths([[1, 2, 3, 4], [5, 6]])
  assert x.tolist() == [[1, 2, 3], [5, 6, 0]] and y.tolist() == [[2, 3, 4], [6, 0, 0]]
  assert ln.tolist() == [3, 1]
  train, valid, test = load_dataset(preprocess=lambda s: [ord(c) for c in s])
  assert len(train) == 1000 and len(valid) == 100 and len(test) == 100
  b1 = [b[0].shape for b in iterate_batches(train, 8, train=True, seed=1)]
  assert len(b1) == 125
  b2 = [b[0].shape for b in iterate_batches(train, 8, train=True, seed=1)]
  assert b1 == b2  # seeded shuffle is reproducible


# ---------------------------------------------------------------- tokenizers
def test_tokenizers_offline():
  from xotorch_support_jetson_amd.inference.tokenizers import ByteTokenizer, DummyTokenizer
  bt = ByteTokenizer()
  ids = bt.encode("héllo")
  assert bt.decode(ids) == "héllo"
  s = bt.apply_chat_template([{"role": "user", "content": "hi"}], tokenize=False, add_generation_prompt=True)
  assert "hi" in s
  dt = DummyTokenizer()
  assert dt.eos_token_id == 69
  assert isinstance(dt.decode(dt.encode("abc")), str)


# ---------------------------------------------------------------- manual discovery config
def test_network_topology_config(tmp_path):
  from xotorch_support_jetson_amd.networking.manual.network_topology_config import NetworkTopology
  good = {"peers": {"node1": {"address": "127.0.0.1", "port": 50051, "device_capabilities": {
    "model": "MI355X", "chip": "AMD Instinct MI355X", "memory": 294912, "flops": {"fp32": 157.3, "fp16": 2516.6,
                                                                                  "int8": 5033.2}}}}}
  p = tmp_path / "good.json"
  p.write_text(json.dumps(good))
  t = NetworkTopology.from_path(str(p))
  assert t.peers["node1"].port == 50051 and t.peers["node1"].device_capabilities.memory == 294912
  bad = tmp_path / "bad.json"
  bad.write_text("{not json")
  with pytest.raises(ValueError, match="invalid JSON"):
    NetworkTopology.from_path(str(bad))
  missing = tmp_path / "missing_field.json"
  missing.write_text(json.dumps({"peers": {"n": {"address": "x"}}}))
  with pytest.raises(ValueError):
    NetworkTopology.from_path(str(missing))
  with pytest.raises(FileNotFoundError):
    NetworkTopology.from_path(str(tmp_path / "nope.json"))


def test_stream_chunks_match_generate_completion():
  """The streaming fast path encodes chunks byte-identical to json.dumps(generate_completion(...))."""
  import json as _json
  from unittest import mock

  from xotorch_support_jetson_amd.api.chatgpt_api import (ChatCompletionRequest, Message, StreamChunks,
                                                           generate_completion)
  from xotorch_support_jetson_amd.inference.tokenizers import _resolve_tokenizer

  tok = _resolve_tokenizer("byte", 512)
  req = ChatCompletionRequest("llama-3.2-1b", [Message("user", "hi")], 0.6)
  enc = StreamChunks(req, tok, "rid-1")
  with mock.patch("time.time", return_value=1700000000.5):
    for toks, fr in (([72, 105], None), ([], "length"), ([34, 92, 10], "stop"), ([0xe4, 0xbd, 0xa0], None)):
      want = "data: " + _json.dumps(generate_completion(req, tok, "p", "rid-1", toks, True, fr,
                                                        "chat.completion.chunk")) + "\n\n"
      assert enc.line(toks, fr) == want.encode()


def test_direct_sse_framing_and_fallback():
  """Direct SSE writes: each token's chunk is HTTP/1.1-chunk framed onto the transport; a slow reader (full
  socket buffer) sends the stream back to the queue path without losing or reordering tokens."""
  import asyncio as _asyncio

  from xotorch_support_jetson_amd.api import chatgpt_api as ca
  from xotorch_support_jetson_amd.inference.tokenizers import _resolve_tokenizer

  class FakeTransport:
    def __init__(self):
      self.out, self.buffered = [], 0

    def write(self, b):
      self.out.append(b)

    def is_closing(self):
      return False

    def get_write_buffer_size(self):
      return self.buffered

  async def main():
    tok = _resolve_tokenizer("byte", 512)
    req = ca.ChatCompletionRequest("m", [ca.Message("user", "x")], 0.0)
    chunks = ca.StreamChunks(req, tok, "r")
    api = ca.ChatGPTAPI.__new__(ca.ChatGPTAPI)  # only the token fan-in state
    api.token_queues, api._direct = {"r": _asyncio.Queue()}, {}
    t = FakeTransport()
    d = ca._DirectStream(t, chunks, {2}, None, lambda: None)
    api._direct["r"] = d
    api.handle_tokens("r", [72], False)
    api.handle_tokens("r", [105], False)
    line = chunks.line([72], None)
    assert t.out[0] == b"%x\r\n" % len(line) + line + b"\r\n"
    assert len(t.out) == 2 and api.token_queues["r"].empty()
    t.buffered = ca.DIRECT_SSE_MAX_BUFFER + 1  # the reader stalls
    api.handle_tokens("r", [33], False)
    api.handle_tokens("r", [2], True)
    assert d.fallback and d.done.done() and "r" not in api._direct and len(t.out) == 2
    q = api.token_queues["r"]
    assert [q.get_nowait(), q.get_nowait()] == [([33], False), ([2], True)]

  _asyncio.run(main())


def test_gemm_policy_table_persists(tmp_path, monkeypatch):
  """Tuned GEMM choices round-trip through the on-disk table (tuples restored, atomic writes), and a new
  policy object starts from it instead of re-timing."""
  from xotorch_support_jetson_amd.ops import linear as L

  path = tmp_path / "g" / "table.json"
  monkeypatch.setenv("XOT_GEMM_TABLE", str(path))
  p = L.GemmPolicy()
  key = ("sh", 512, 8192, 8192, "resid", False, "torch.bfloat16")
  assert p._lookup(key) is None
  p._store(key, ("big", 128, 2))
  p._store(("rm", 1, 64, 64, "none", False), "blas")
  assert path.exists() and not list(path.parent.glob("*.tmp"))
  q = L.GemmPolicy()
  assert q._lookup(key) == ("big", 128, 2)
  assert q._lookup(("rm", 1, 64, 64, "none", False)) == "blas"
  path.write_text("{not json")
  assert L.GemmPolicy()._lookup(key) is None  # a corrupt table is ignored
  monkeypatch.setenv("XOT_GEMM_TABLE", "off")
  assert L._default_table_path() is None


def test_gemm_row_tiles_for_unaligned_batches():
  """Decode batches between the 256-row multiples get shorter row tiles (no 32+ padding rows per tile) as
  extra timed candidates, and their tuning keys no longer collapse onto the next power of two."""
  from xotorch_support_jetson_amd.ops import linear as L
  assert [L.big_row_tile(m) for m in (1, 256, 300, 320, 384, 448, 480, 512, 576, 700)] == \
      [160, 256, 160, 160, 192, 224, 256, 256, 192, 256]
  assert [L._m_bucket(m) for m in (1, 200, 256, 300, 448, 512, 1000, 1500, 5000)] == \
      [1, 256, 256, 320, 448, 512, 1024, 2048, 8192]
  cands = L.GemmPolicy._big_cands(448, 8192, 8192)
  assert ("big", 2240256, 1) in cands and ("big", 2240128, 2) in cands
  assert all(L.tile_rows(c[1]) == 256 for c in L.GemmPolicy._big_cands(512, 8192, 8192) if c[0] == "big")
  assert L.tile_width(2240128) == 128 and L.tile_rows(2240128) == 224 and L.tile_rows(1256) == 256
  h = L.GemmPolicy._heuristic(384, 57344, L.GemmPolicy._big_cands(384, 57344, 8192))
  assert h[0] == "big", h  # (untuned fallback; the timed choice decides between 256- and 192-row tiles)


def test_pmc_summary_decode_window(tmp_path):
  """tools/pmc_summary.py joins the counter passes of a pmc.sh run per (kernel, grid) over the last decode
  steps only (delimited by the sampler), so tuning calls before them never mix into the rates."""
  import csv
  import subprocess
  import sys
  fields = ["Dispatch_Id", "Kernel_Name", "Grid_Size", "Counter_Name", "Counter_Value", "Start_Timestamp",
            "End_Timestamp"]
  for p, ctr, val in (("p1", "GRBM_GUI_ACTIVE", 8e6), ("p2", "SQ_VALU_MFMA_BUSY_CYCLES", 5e8)):
    d = tmp_path / p / "host"
    d.mkdir(parents=True)
    with open(d / "1_p_counter_collection.csv", "w", newline="") as f:
      w = csv.DictWriter(f, fieldnames=fields)
      w.writeheader()
      t = 0
      seq = [("gemm_big_kernel<1>(int)", 999, 1.0)] * 3  # tuning calls: another grid, another rate
      seq += [("gemm_big_kernel<1>(int)", 512, 1.0), ("attn(int)", 64, 1.0), ("sample_fast_kernel(int)", 1, 1.0)] * 3
      for i, (k, grid, _) in enumerate(seq):
        t += 1_000_000
        v = val if grid != 999 else val / 10
        w.writerow(dict(Dispatch_Id=i, Kernel_Name=k, Grid_Size=grid, Counter_Name=ctr, Counter_Value=v,
                        Start_Timestamp=t, End_Timestamp=t + 500_000))
  out = tmp_path / "s.json"
  tool = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "pmc_summary.py")
  subprocess.run([sys.executable, tool, str(tmp_path), "--window", "sample_fast_kernel", "--last", "2",
                  "--match", "gemm_big", "--json", str(out)], check=True, capture_output=True)
  s = json.loads(out.read_text())
  assert list(s) == ["gemm_big_kernel<1> grid=512"]
  r = s["gemm_big_kernel<1> grid=512"]
  assert r["us"] == 500.0 and r["clock_ghz"] == 2.0 and r["mfma_busy_pct"] == 48.8

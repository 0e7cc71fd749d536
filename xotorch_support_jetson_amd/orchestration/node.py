"""Node: one peer of the ring (reference: xotorch/orchestration/node.py:22-611).

Owns the peers, the topology, one inference engine (holding this peer's layer shard) and the
per-request bookkeeping.  Requests circulate first shard -> ... -> last shard (samples) -> first
shard, one ring trip per generated token.

Behaviour kept from the reference: ring memory-weighted partitioning recomputed from the live
topology on every request, opaque-status JSON messages (start/end_process_prompt, train/eval example,
download_progress, supported_inference_engines), topology gossip every 2 s, pipeline training with the
input-gradient returned in the SendExample reply, per-shard checkpoints every N iterations.
Fixed by design (each is a test): the API temperature / max_tokens reach the sampler
(node.py:121 ignores them); token results go to the requesting peer only, not to every peer per
token (node.py:580-591); finished requests free their token buffers and every peer's KV pages
(node.py:117-147 never frees); a peer change does not replace the engine and drop the loaded model
(node.py:513-518); checkpoint names are deterministic (node.py:238 uses the salted hash()).
"""
from __future__ import annotations

import asyncio
import json
import time
import traceback
import uuid
from typing import Dict, List, Optional, Tuple

import numpy as np

from ..helpers import DEBUG, AsyncCallbackSystem
from ..inference.inference_engine import InferenceEngine, get_inference_engine
from ..inference.shard import Shard
from ..networking import Discovery, PeerHandle, Server
from ..topology.device_capabilities import UNKNOWN_DEVICE_CAPABILITIES, DeviceCapabilities, device_capabilities
from ..topology.partitioning_strategy import Partition, PartitioningStrategy, map_partitions_to_shards
from ..topology.topology import Topology
from .tracing import tracer


class Node:
  def __init__(self, _id: str, server: Optional[Server], inference_engine: InferenceEngine, discovery: Discovery,
               shard_downloader, partitioning_strategy: PartitioningStrategy, max_generate_tokens: int = 1024,
               default_sample_temperature: float = 0.0, topology_viz=None,
               device_caps: Optional[DeviceCapabilities] = None):
    self.id = _id
    self.server = server
    self.inference_engine = inference_engine
    self.discovery = discovery
    self.shard_downloader = shard_downloader
    self.partitioning_strategy = partitioning_strategy
    self.peers: List[PeerHandle] = []
    self.topology: Topology = Topology()
    self.device_capabilities = device_caps or UNKNOWN_DEVICE_CAPABILITIES
    self._caps_override = device_caps
    self.buffered_token_output: Dict[str, Tuple[List[int], bool]] = {}
    self.request_params: Dict[str, dict] = {}  # temperature / top_k / max_tokens per request
    self.request_origin: Dict[str, str] = {}  # request id -> node id that owns the API call
    self.max_generate_tokens = max_generate_tokens
    self.default_sample_temperature = default_sample_temperature
    self.topology_viz = topology_viz
    self.outstanding_requests: Dict[str, str] = {}
    self.checkpoints: Dict[str, Dict[str, List[int]]] = {}
    self.node_download_progress: Dict[str, dict] = {}
    self.topology_inference_engines_pool: List[List[str]] = []
    self._on_token = AsyncCallbackSystem[str, Tuple[str, List[int], bool]]()
    self._on_opaque_status = AsyncCallbackSystem[str, Tuple[str, str]]()
    self._on_opaque_status.register("node_status").on_next(self.on_node_status)
    self._tasks: List[asyncio.Task] = []
    self.token_count = 0
    self.first_token_time = 0.0

  # ------------------------------------------------------------------ lifecycle
  async def start(self, wait_for_peers: int = 0) -> None:
    self.device_capabilities = self._caps_override or device_capabilities()
    if self.server is not None:
      await self.server.start()
    await self.discovery.start()
    await self.update_peers(wait_for_peers)
    await self.collect_topology(set())
    if DEBUG >= 2:
      print(f"Collected topology: {self.topology}")
    self._tasks.append(asyncio.create_task(self.periodic_topology_collection(2.0)))

  async def stop(self) -> None:
    for t in self._tasks:
      t.cancel()
    await asyncio.gather(*self._tasks, return_exceptions=True)
    await self.discovery.stop()
    if self.server is not None:
      await self.server.stop()

  # ------------------------------------------------------------------ status messages
  def on_node_status(self, request_id, opaque_status):
    try:
      status = json.loads(opaque_status)
      kind = status.get("type")
      if kind == "supported_inference_engines":
        self.topology_inference_engines_pool.append(status.get("engines", []))
      elif kind == "node_status":
        st = status.get("status", "")
        if st.startswith("start_"):
          self.current_topology.active_node_id = status.get("node_id")
          if st == "start_process_prompt" and status.get("origin"):
            self.request_origin.setdefault(status.get("request_id"), status["origin"])
        elif st.startswith("end_"):
          if status.get("node_id") == self.current_topology.active_node_id:
            self.current_topology.active_node_id = None
        elif st == "request_finished":
          rid = status.get("request_id")
          asyncio.get_running_loop().create_task(self._release_request(rid, ok=not status.get("failed")))
      elif kind == "save_checkpoint" and status.get("node_id") != self.id:
        asyncio.get_running_loop().create_task(self.coordinate_save(
          Shard.from_dict(status["base_shard"]), int(status["iteration"]), status["destination"], broadcast=False))
      elif kind == "download_progress":
        self.node_download_progress[status.get("node_id")] = status.get("progress")
      if self.topology_viz:
        self.topology_viz.update_visualization(self.topology, self.partitioning_strategy.partition(self.topology), self.id,
                                               self.node_download_progress, num_layers=self._viz_layers())
    except Exception as e:
      if DEBUG >= 1:
        print(f"Error on_node_status: {e}")
        traceback.print_exc()

  async def _release_request(self, request_id: Optional[str], ok: bool = True) -> None:
    """Free a finished request's engine state.  ok=False: it was aborted or failed part-way (a hop to a dead
    peer, a failed decode step), so its steps may not have reached every shard -- the engine must not
    treat what it started for the request (a prefix-cache save) as applied ring-wide."""
    if not request_id:
      return
    self.request_params.pop(request_id, None)
    self.outstanding_requests.pop(request_id, None)
    try:
      await self.inference_engine.finish_request(request_id, ok=ok)
    except Exception:
      if DEBUG >= 2:
        traceback.print_exc()
    # keep the buffered output a little while for late API readers, then drop it
    await asyncio.sleep(30)
    self.buffered_token_output.pop(request_id, None)
    self.request_origin.pop(request_id, None)

  async def broadcast_supported_engines(self, names: List[str]):
    await self.broadcast_opaque_status("", json.dumps({"type": "supported_inference_engines", "node_id": self.id,
                                                       "engines": names}))

  def get_topology_inference_engines(self) -> List[List[str]]:
    return self.topology_inference_engines_pool

  # ------------------------------------------------------------------ inference
  def _params(self, request_id: str, inference_state: Optional[dict]) -> dict:
    p = self.request_params.get(request_id)
    if p is None:
      p = {}
      if inference_state:
        for k in ("temperature", "top_k", "max_tokens"):
          if inference_state.get(k) is not None:
            p[k] = inference_state[k]
      self.request_params[request_id] = p
    return p

  def _norm_sampling(self, state: dict) -> dict:
    """Sampling keys the API sends as None when the client leaves them out (chatgpt_api.py) are filled
    with the node defaults here, once, before the state reaches any engine or peer: the engines read
    `state["temperature"]` as a number."""
    if "temperature" in state and state["temperature"] is None:
      state["temperature"] = self.default_sample_temperature
    for k in ("top_k", "max_tokens"):
      if k in state and state[k] is None:
        del state[k]
    return state

  def _max_tokens(self, params: dict) -> int:
    return min(int(params.get("max_tokens") or self.max_generate_tokens), self.max_generate_tokens)

  def _eos_ids(self) -> set:
    eos = set(getattr(self.inference_engine, "eos_token_ids", ()) or ())
    tk = getattr(self.inference_engine, "tokenizer", None)
    if tk is not None and getattr(tk, "eos_token_id", None) is not None:
      eos.add(int(tk.eos_token_id))
    return eos

  def _emit_token(self, request_id: str, tok: int, max_tokens: int, eos: set) -> bool:
    """Record one sampled token of a request on its last shard: buffer, token callbacks, result broadcast,
    and the end of the request.  Returns whether the request is finished."""
    buf = self.buffered_token_output.setdefault(request_id, ([], False))
    buf[0].append(tok)
    is_finished = tok in eos or len(buf[0]) >= max_tokens
    if DEBUG >= 2:
      print(f"[{request_id}] token {tok} finished={is_finished} n={len(buf[0])}")
    self.trigger_on_token_callbacks(request_id, [tok], is_finished)
    if self.peers:
      asyncio.create_task(self.broadcast_result(request_id, [tok], is_finished))
    if is_finished:
      self._finish(request_id)
    return is_finished

  def _finish(self, request_id: str, failed: bool = False) -> None:
    buf = self.buffered_token_output.setdefault(request_id, ([], False))
    self.buffered_token_output[request_id] = (buf[0], True)
    self.outstanding_requests.pop(request_id, None)
    status = {"type": "node_status", "node_id": self.id, "status": "request_finished", "request_id": request_id}
    if failed:
      status["failed"] = True
    asyncio.create_task(self.broadcast_opaque_status(request_id, json.dumps(status)))

  def _abort(self, request_id: str) -> None:
    """A request the engine's decode loop could not continue: its consumers (API streams, CLI) get the end
    of the request now -- with only _finish they would wait for a token that never comes."""
    self.trigger_on_token_callbacks(request_id, [], True)
    if self.peers:
      asyncio.create_task(self.broadcast_result(request_id, [], True))
    self._finish(request_id, failed=True)

  async def process_inference_result(self, shard: Shard, result, request_id: Optional[str] = None,
                                     inference_state: Optional[dict] = None):
    params = self._params(request_id, inference_state)
    max_tokens = self._max_tokens(params)
    buf = self.buffered_token_output.setdefault(request_id, ([], False))
    is_finished = len(buf[0]) >= max_tokens
    forward = result
    if shard.is_last_layer() and not is_finished:
      temp = params.get("temperature")
      temp = self.default_sample_temperature if temp is None else float(temp)
      token = await self.inference_engine.sample(result, temp=temp, top_k=int(params.get("top_k") or 35))
      tok = int(np.asarray(token).reshape(-1)[0])
      eos = self._eos_ids()
      is_finished = self._emit_token(request_id, tok, max_tokens, eos)
      forward = np.asarray([[tok]], dtype=np.int64)
      if not is_finished and shard.is_first_layer():
        # this peer holds the whole model: hand the request to the engine's decode loop, which runs its next
        # steps back to back and reports each token here (no per-token coroutine chain through the Node)
        loop = getattr(self.inference_engine, "continue_locally", None)
        state = dict(inference_state or {})
        state.update(params)
        if state.get("temperature") is None:
          state["temperature"] = temp
        def stop(rid: str, t: int) -> bool:  # would _emit_token(rid, t) end the request? (no side effects)
          return t in eos or len(self.buffered_token_output.get(rid, ((),))[0]) + 1 >= max_tokens
        if loop is not None and loop(request_id, shard, tok, state,
                                     lambda rid, t: self._emit_token(rid, t, max_tokens, eos), self._abort,
                                     stop=stop):
          self.outstanding_requests[request_id] = "processing"
          return np.array(buf[0])
    elif shard.is_last_layer():  # already at max_tokens
      self.trigger_on_token_callbacks(request_id, [], True)
      if self.peers:
        asyncio.create_task(self.broadcast_result(request_id, [], True))
      self._finish(request_id)
    if is_finished:
      self.buffered_token_output[request_id] = (buf[0], True)
      self.outstanding_requests.pop(request_id, None)
    else:
      self.outstanding_requests[request_id] = "waiting"
      state = dict(inference_state or {})
      state.update({k: v for k, v in params.items()})
      asyncio.create_task(self.forward_tensor(shard, forward, request_id, self.get_partition_index(offset=1), state))
    return np.array(buf[0])

  async def process_prompt(self, base_shard: Shard, prompt: str, request_id: Optional[str] = None,
                           inference_state: Optional[dict] = None) -> None:
    if request_id is None:
      request_id = str(uuid.uuid4())
    shard = self.get_current_shard(base_shard)
    origin = (inference_state or {}).get("origin") or self.id
    self.request_origin.setdefault(request_id, origin)
    state = self._norm_sampling(dict(inference_state or {}))
    state["origin"] = origin
    self._params(request_id, state)
    asyncio.create_task(self.broadcast_opaque_status(request_id, json.dumps({
      "type": "node_status", "node_id": self.id, "status": "start_process_prompt", "base_shard": base_shard.to_dict(),
      "shard": shard.to_dict(), "prompt": prompt, "request_id": request_id, "origin": origin})))
    t0 = time.perf_counter_ns()
    with tracer.span("process_prompt", request_id=request_id, node=self.id):
      await self._process_prompt(base_shard, prompt, request_id, state)
    elapsed = time.perf_counter_ns() - t0
    asyncio.create_task(self.broadcast_opaque_status(request_id, json.dumps({
      "type": "node_status", "node_id": self.id, "status": "end_process_prompt", "base_shard": base_shard.to_dict(),
      "shard": shard.to_dict(), "prompt": prompt, "request_id": request_id, "elapsed_time_ns": elapsed})))
    if DEBUG >= 2:
      print(f"[{request_id}] process prompt: {base_shard=} {shard=} {elapsed=}")

  async def _process_prompt(self, base_shard: Shard, prompt: str, request_id: str,
                            inference_state: Optional[dict] = None):
    shard = self.get_current_shard(base_shard)
    if not shard.is_first_layer():
      self.outstanding_requests[request_id] = "waiting"
      await self.forward_prompt(shard, prompt, request_id, 0, inference_state)
      return None
    self.outstanding_requests[request_id] = "processing"
    result, state = await self.inference_engine.infer_prompt(request_id, shard, prompt, inference_state)
    state = {**(inference_state or {}), **(state or {})}
    await self.process_inference_result(shard, result, request_id, state)
    return result

  async def process_tensor(self, base_shard: Shard, tensor, request_id: Optional[str] = None,
                           inference_state: Optional[dict] = None):
    shard = self.get_current_shard(base_shard)
    t0 = time.perf_counter_ns()
    resp = await self._process_tensor(shard, tensor, request_id, inference_state)
    if DEBUG >= 2:
      print(f"[{request_id}] process_tensor {shard} {(time.perf_counter_ns() - t0) / 1e6:.2f} ms")
    return resp

  async def _process_tensor(self, base_shard: Shard, tensor, request_id: Optional[str] = None,
                            inference_state: Optional[dict] = None):
    if request_id is None:
      request_id = str(uuid.uuid4())
    shard = self.get_current_shard(base_shard)
    if inference_state and inference_state.get("origin"):
      self.request_origin.setdefault(request_id, inference_state["origin"])
    self._params(request_id, inference_state)
    try:
      self.outstanding_requests[request_id] = "processing"
      result, state = await self.inference_engine.infer_tensor(request_id, shard, tensor, inference_state)
      state = {**(inference_state or {}), **(state or {})}
      return await self.process_inference_result(shard, result, request_id, state)
    except Exception as e:
      self.outstanding_requests.pop(request_id, None)
      print(f"Error processing tensor for shard {shard}: {e}")
      traceback.print_exc()

  # ------------------------------------------------------------------ training
  async def enqueue_example(self, base_shard: Shard, example, target, length, request_id: Optional[str] = None,
                            train: bool = False):
    shard = self.get_current_shard(base_shard)
    if shard.is_first_layer():
      return await self.process_example(shard, example, target, length, train, request_id)
    if request_id is None:
      request_id = str(uuid.uuid4())
    self.outstanding_requests[request_id] = "waiting"
    return await self.forward_example(shard, example, target, length, train, request_id, 0)

  async def coordinate_save(self, base_shard: Shard, iteration: int, destination: str, broadcast: bool = True):
    """Save this peer's shard and (broadcast=True) tell every other peer to save theirs, so a ring
    checkpoint covers all layers (the reference saves only the calling peer's shard, node.py:230-252)."""
    if broadcast:
      await self.broadcast_opaque_status("", json.dumps({
        "type": "save_checkpoint", "node_id": self.id, "base_shard": base_shard.to_dict(), "iteration": iteration,
        "destination": destination}))
    from ..train.checkpoint import checkpoint_path
    shard = self.get_current_shard(base_shard)
    model, sid = shard.model_id, shard.key()
    key = f"{sid}::{iteration}"
    self.outstanding_requests[key] = "Checking"
    done = self.checkpoints.setdefault(model, {}).setdefault(sid, [])
    try:
      if not done or done[-1] < iteration:
        path = checkpoint_path(destination, shard, iteration)
        print(f"Saving checkpoint to {path}")
        self.outstanding_requests[key] = "Saving"
        path.parent.mkdir(parents=True, exist_ok=True)
        await self.inference_engine.save_checkpoint(shard, str(path))
        self.checkpoints[model][sid] = sorted(done + [iteration])
    finally:
      self.outstanding_requests.pop(key, None)

  async def process_example(self, base_shard: Shard, example, target, length, train: bool = False,
                            request_id: Optional[str] = None):
    shard = self.get_current_shard(base_shard)
    kind = "train" if train else "eval"
    # (a downstream stage's example is a bf16 activation tensor, which numpy cannot hold)
    shape = [int(d) for d in (example.shape if hasattr(example, "shape") else np.asarray(example).shape)]
    asyncio.create_task(self.broadcast_opaque_status(request_id, json.dumps({
      "type": "node_status", "node_id": self.id, "status": f"start_{kind}_example", "base_shard": base_shard.to_dict(),
      "shard": shard.to_dict(), "example_size": int(np.prod(shape)), "example_shape": shape,
      "request_id": request_id})))
    t0 = time.perf_counter_ns()
    resp = await self._process_example(shard, example, target, length, train, request_id)
    asyncio.create_task(self.broadcast_opaque_status(request_id, json.dumps({
      "type": "node_status", "node_id": self.id, "status": f"end_{kind}_example", "base_shard": base_shard.to_dict(),
      "shard": shard.to_dict(), "request_id": request_id, "elapsed_time_ns": time.perf_counter_ns() - t0})))
    return resp

  async def _process_example(self, base_shard: Shard, example, target, length, train: bool = False,
                             request_id: Optional[str] = None):
    if request_id is None:
      request_id = str(uuid.uuid4())
    shard = self.get_current_shard(base_shard)
    eng = self.inference_engine
    try:
      target = np.asarray(target).astype(np.int64)
      if train:
        if shard.is_last_layer():
          self.outstanding_requests[request_id] = "training"
          loss, grad = await eng.train(request_id, shard, example, target, length)
        else:
          self.outstanding_requests[request_id] = "preprocessing"
          fwd = getattr(eng, "train_forward", None)
          step = await fwd(request_id, shard, example) if fwd else (await eng.infer_tensor(request_id, shard, example))[0]
          self.outstanding_requests[request_id] = "waiting"
          loss, backgrad = await self.forward_example(shard, step, target, length, train, request_id,
                                                      self.get_partition_index(offset=1))
          self.outstanding_requests[request_id] = "training"
          _, grad = await eng.train(request_id, shard, example, backgrad, length, loss="back_gradient")
        self.outstanding_requests.pop(request_id, None)
        return loss if shard.is_first_layer() else (loss, grad)
      if shard.is_last_layer():
        self.outstanding_requests[request_id] = "evaluating"
        loss = await eng.evaluate(request_id, shard, example, target, length)
      else:
        self.outstanding_requests[request_id] = "preprocessing"
        fwd = getattr(eng, "eval_forward", None)
        step = await fwd(request_id, shard, example) if fwd else (await eng.infer_tensor(request_id, shard, example))[0]
        self.outstanding_requests[request_id] = "waiting"
        loss = await self.forward_example(shard, step, target, length, train, request_id,
                                          self.get_partition_index(offset=1))
      self.outstanding_requests.pop(request_id, None)
      return loss
    except Exception as e:
      self.outstanding_requests.pop(request_id, None)
      print(f"Error processing example for shard {shard}: {e}")
      traceback.print_exc()
      return None

  # ------------------------------------------------------------------ ring forwarding
  async def forward_example(self, base_shard: Shard, step, target, length, train: bool, request_id: str,
                            target_index: int):
    target_id = self._partition_node(target_index)
    target_shard = self.get_current_shard(base_shard, target_index)
    if target_id == self.id:
      return await self.process_example(target_shard, step, target, length, train, request_id)
    peer = self._peer(target_id)
    return await peer.send_example(target_shard, step, target, length, train=train, request_id=request_id)

  async def forward_prompt(self, base_shard: Shard, prompt: str, request_id: str, target_index: int,
                           inference_state: Optional[dict] = None):
    target_id = self._partition_node(target_index)
    next_shard = self.get_current_shard(base_shard, target_index)
    if target_id == self.id:
      return await self.process_prompt(next_shard, prompt, request_id, inference_state)
    try:
      await self._peer(target_id).send_prompt(next_shard, prompt, request_id=request_id,
                                              inference_state=inference_state)
    except Exception as e:
      await self._fail_request(request_id, target_id, e)

  async def forward_tensor(self, base_shard: Shard, tensor, request_id: str, target_index: int,
                           inference_state: Optional[dict] = None):
    target_id = self._partition_node(target_index)
    next_shard = self.get_current_shard(base_shard, target_index)
    if target_id == self.id:
      return await self.process_tensor(next_shard, tensor, request_id, inference_state)
    try:
      with tracer.span("hop", request_id=request_id, to=target_id):
        await self._peer(target_id).send_tensor(next_shard, tensor, request_id=request_id,
                                                inference_state=inference_state)
    except Exception as e:
      await self._fail_request(request_id, target_id, e)

  async def _fail_request(self, request_id: str, peer_id: str, err: Exception) -> None:
    """A hop to `peer_id` failed (peer gone or unreachable): the request cannot continue because that
    peer holds part of its KV cache.  Finish it at its origin (the API answers with the tokens so far
    instead of hanging until its timeout), free its pages on the live peers, and refresh peers and
    topology so the next request is re-partitioned over the peers that are still up (the reference
    logs the error and leaves the request hanging, node.py:424-443)."""
    print(f"Error forwarding {request_id} to {peer_id}: {err}; finishing the request and re-partitioning")
    self.outstanding_requests.pop(request_id, None)
    origin = self.request_origin.get(request_id) or self.id
    buf = self.buffered_token_output.get(request_id, ([], False))
    self.buffered_token_output[request_id] = (buf[0], True)
    if origin == self.id:
      self.trigger_on_token_callbacks(request_id, [], True)
    else:
      try:
        await asyncio.wait_for(self._peer(origin).send_result(request_id, [], True), timeout=5.0)
      except Exception:
        pass
    dead = [p for p in self.peers if p.id() == peer_id]
    self.peers = [p for p in self.peers if p.id() != peer_id]
    for p in dead:
      try:
        await asyncio.wait_for(p.disconnect(), timeout=2.0)
      except Exception:
        pass
    try:
      await self.collect_topology(set())
    except Exception:
      pass
    asyncio.create_task(self.broadcast_opaque_status(request_id, json.dumps(
      {"type": "node_status", "node_id": self.id, "status": "request_finished", "request_id": request_id,
       "failed": True})))

  def _peer(self, node_id: str) -> PeerHandle:
    for p in self.peers:
      if p.id() == node_id:
        return p
    raise ValueError(f"Peer for {node_id} not found")

  def _partitions(self) -> List[Partition]:
    """Partitions of the current topology, memoised per topology content: every generated token asks
    several times (shard of this peer, next hop), and the topology only changes on gossip."""
    topo = self.topology
    key = (id(topo), tuple(sorted((nid, caps.memory) for nid, caps in topo.nodes.items())))
    cached = getattr(self, "_parts_cache", None)
    if cached is not None and cached[0] == key:
      return cached[1]
    parts = self.partitioning_strategy.partition(topo)
    self._parts_cache = (key, parts)
    return parts

  def _partition_node(self, index: int) -> str:
    parts = self._partitions()
    return parts[index % len(parts)].node_id

  def get_partition_index(self, offset: int = 0) -> int:
    if not self.partitioning_strategy:
      return 0
    parts = self._partitions()
    idx = next((i for i, p in enumerate(parts) if p.node_id == self.id), None)
    if idx is None:
      raise ValueError(f"No current partition found for node: {self.id}")
    return (idx + offset) % len(parts)

  def get_current_shard(self, base_shard: Shard, index: Optional[int] = None) -> Shard:
    if index is None:
      index = self.get_partition_index()
    shards = map_partitions_to_shards(self._partitions(), base_shard.n_layers, base_shard.model_id)
    return shards[index % len(shards)]

  # ------------------------------------------------------------------ peers / topology
  async def update_peers(self, wait_for_peers: int = 0) -> bool:
    next_peers = await self.discovery.discover_peers(wait_for_peers)
    cur = {p.id(): p for p in self.peers}
    nxt = {p.id(): p for p in next_peers}
    removed = [p for pid, p in cur.items() if pid not in nxt]
    added = [p for pid, p in nxt.items() if pid not in cur]
    updated = [p for pid, p in nxt.items() if pid in cur and p.addr() != cur[pid].addr()]
    unchanged = [p for pid, p in nxt.items() if pid in cur and p.addr() == cur[pid].addr()]

    async def _disconnect(p):
      try:
        await asyncio.wait_for(p.disconnect(), timeout=5)
      except Exception:
        pass

    async def _connect(p):
      try:
        await asyncio.wait_for(p.connect(), timeout=5)
        return True
      except Exception:
        return False

    await asyncio.gather(*(_disconnect(p) for p in removed), *(_disconnect(cur[p.id()]) for p in updated))
    oks = await asyncio.gather(*(_connect(p) for p in added + updated))
    connected = [p for p, ok in zip(added + updated, oks) if ok]
    self.peers = unchanged + connected
    changed = bool(removed or added or updated)
    if changed and DEBUG >= 1:
      print(f"peers changed: +{[p.id() for p in added]} -{[p.id() for p in removed]} ~{[p.id() for p in updated]}")
    return changed

  async def periodic_topology_collection(self, interval: float):
    while True:
      await asyncio.sleep(interval)
      try:
        await self.update_peers()
        await self.collect_topology(set())
      except Exception as e:
        if DEBUG >= 1:
          print(f"Error collecting topology: {e}")

  async def collect_topology(self, visited: set, max_depth: int = 4) -> Topology:
    next_topology = Topology()
    next_topology.update_node(self.id, self.device_capabilities)
    visited = set(visited) | {self.id}
    for p in self.peers:
      if max_depth > 0 and p.id() not in visited:
        try:
          other = await asyncio.wait_for(p.collect_topology(visited | {p.id()}, max_depth - 1), timeout=5.0)
        except Exception as e:
          # an unreachable peer leaves the topology (and so the partitioning) until discovery and a
          # successful collection bring it back
          if DEBUG >= 2:
            print(f"Error collecting topology from {p.id()}: {e}")
          continue
        next_topology.update_node(p.id(), p.device_capabilities())
        next_topology.add_edge(self.id, p.id(), p.description())
        next_topology.merge(p.id(), other)
        visited.add(p.id())
      else:
        next_topology.update_node(p.id(), p.device_capabilities())
        next_topology.add_edge(self.id, p.id(), p.description())
    next_topology.active_node_id = self.topology.active_node_id
    self.topology = next_topology
    if self.topology_viz:
      self.topology_viz.update_visualization(self.topology, self._partitions(), self.id, num_layers=self._viz_layers())
    return self.topology

  def _viz_layers(self):
    """Layer count of the model this node serves (the TUI shows each peer's layer range), if one is loaded."""
    shard = getattr(self.inference_engine, "shard", None)
    return getattr(shard, "n_layers", None)

  @property
  def current_topology(self) -> Topology:
    return self.topology

  def layer_ranges(self):
    """[(peer id, first layer, last layer)] of the current partitioning for the loaded model (empty if none)."""
    L = self._viz_layers()
    if not L:
      return []
    from ..topology.partitioning_strategy import map_partitions_to_shards
    parts = self._partitions()
    shards = map_partitions_to_shards(parts, L, "m")
    if len(shards) != len(parts):  # a peer without layers: ranges would not line up with the peers
      return []
    return [(p.node_id, s.start_layer, s.end_layer) for p, s in zip(parts, shards)]

  # ------------------------------------------------------------------ callbacks / broadcast
  @property
  def on_token(self) -> AsyncCallbackSystem[str, Tuple[str, List[int], bool]]:
    return self._on_token

  @property
  def on_opaque_status(self) -> AsyncCallbackSystem[str, Tuple[str, str]]:
    return self._on_opaque_status

  def trigger_on_token_callbacks(self, request_id: str, tokens: List[int], is_finished: bool) -> None:
    self.on_token.trigger_all(request_id, tokens, is_finished)

  async def broadcast_result(self, request_id: str, result: List[int], is_finished: bool) -> None:
    origin = self.request_origin.get(request_id)
    targets = [p for p in self.peers if origin is None or p.id() == origin]

    async def send(p):
      try:
        await asyncio.wait_for(p.send_result(request_id, result, is_finished), timeout=15.0)
      except Exception as e:
        if DEBUG >= 2:
          print(f"Error sending result to {p.id()}: {e}")

    await asyncio.gather(*(send(p) for p in targets), return_exceptions=True)

  async def broadcast_opaque_status(self, request_id: str, status: str) -> None:
    async def send(p):
      try:
        await asyncio.wait_for(p.send_opaque_status(request_id, status), timeout=15.0)
      except Exception as e:
        if DEBUG >= 2:
          print(f"Error sending opaque status to {p.id()}: {e}")

    await asyncio.gather(*(send(p) for p in self.peers), return_exceptions=True)
    self.on_opaque_status.trigger_all(request_id, status)  # also deliver to self

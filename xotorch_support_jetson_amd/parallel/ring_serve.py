"""Serving over the local GPU ring: continuous batching with the activation hand-off on RCCL.

The reference serves one request at a time, moving every hop through gRPC with the JSON state
(xotorch/orchestration/node.py:109-147, 403-443; grpc_peer_handle.py:117-136).  Here the GPUs of one
host are the ring peers (one process each) and the data plane is RCCL p2p over xGMI.

  lanes          rank 0 (API, tokenizer, scheduler) splits the running requests into `world` lanes and
                 cycles through them: a lane's next step starts as soon as its previous step's tokens are
                 back, while the other lanes' steps are on the other GPUs -- so the ring stays full, as
                 in bench.py, instead of filling and draining once per round.
  control        each lane step travels the ring ahead of its data as a small header (float64 tensor on the
                 same p2p edges): the step's requests (integer ids) with their new-token counts and
                 temperatures, requests to free, and a stop flag.  Every rank thus knows every shape it
                 will receive; no collective, so no rank waits for the whole ring to drain.
  data plane     stage r receives [T, D] bf16 from r-1, runs its layers, sends to r+1; the last stage
                 samples on device (temperature / top-k 35) and sends the ids [B] int32 back to rank 0
                 (P2PTransport: one communicator per directed edge, so these never queue behind the
                 forward traffic).  Rank 0 receives lane steps' ids in launch order (FIFO per edge).
  KV             each rank holds the paged KV of its own layers for every running request; a finished
                 request is freed on every rank when the next header passes.

`RingServer.submit()` is thread-safe (the asyncio API calls it); tokens come back through `on_token`
callbacks (request_id, [token], is_finished) -- the reference's token callback contract.
"""
from __future__ import annotations

import queue
import threading
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence

import torch
import torch.distributed as dist

from ..ops import kernels as K


@dataclass
class _Req:
  rid: str
  ids: List[int]
  temp: float
  max_tokens: int
  out: List[int] = field(default_factory=list)
  key: int = -1  # integer id on the wire
  lane: int = 0


class RingServer:
  def __init__(self, runner, rank: int, world: int, transport, ctl_group=None, eos_ids: Sequence[int] = (),
               top_k: int = 35, seed: int = 1234, max_batch: Optional[int] = None):
    self.r, self.rank, self.world, self.t = runner, rank, world, transport
    self.ctl = ctl_group  # (unused: the control messages travel with the data)
    self.first, self.last = runner.shard.is_first_layer(), runner.shard.is_last_layer()
    self.prev, self.next = (rank - 1) % world, (rank + 1) % world
    self.D = runner.config.hidden_size
    self.dev = runner.device
    self.eos = set(int(e) for e in eos_ids)
    self.top_k = top_k
    self.seed_off = torch.tensor([seed, 0], dtype=torch.int64, device=runner.device)
    self.max_batch = max_batch or runner.max_batch
    self.lanes = max(1, world)
    self._inbox: "queue.Queue[_Req]" = queue.Queue()
    self._running: Dict[str, _Req] = {}
    self._by_key: Dict[int, _Req] = {}
    self._next_key = 0
    self._free: List[int] = []  # keys to free on every rank (carried by the next header)
    self._inflight: List[Optional[list]] = [None] * self.lanes  # per lane: the step's requests awaiting ids
    self._callbacks: List[Callable[[str, List[int], bool], None]] = []
    self._stop = False
    self._wake = threading.Event()

  # ------------------------------------------------------------------ rank-0 API side
  def submit(self, rid: str, ids: Sequence[int], temp: float = 0.0, max_tokens: int = 256) -> None:
    self._inbox.put(_Req(rid, [int(i) for i in ids], float(temp), int(max_tokens)))
    self._wake.set()

  def on_token(self, cb: Callable[[str, List[int], bool], None]) -> None:
    self._callbacks.append(cb)

  def stop(self) -> None:
    self._stop = True
    self._wake.set()

  def idle(self) -> bool:
    return not self._running and self._inbox.empty()

  def _emit(self, rid: str, toks: List[int], fin: bool) -> None:
    for cb in self._callbacks:
      cb(rid, toks, fin)

  # ------------------------------------------------------------------ wire format
  @staticmethod
  def _header(items, free, stop: bool) -> torch.Tensor:
    """[n_items, n_free, stop, (key, qlen, temp) * n_items, key * n_free] as float64 (exact for ids < 2^53)."""
    vals = [float(len(items)), float(len(free)), 1.0 if stop else 0.0]
    for key, qlen, temp in items:
      vals += [float(key), float(qlen), float(temp)]
    vals += [float(k) for k in free]
    return torch.tensor(vals, dtype=torch.float64)

  @staticmethod
  def _parse(h: torch.Tensor):
    v = h.tolist()
    n, nf, stop = int(v[0]), int(v[1]), v[2] != 0.0
    items = [(int(v[3 + 3 * i]), int(v[4 + 3 * i]), v[5 + 3 * i]) for i in range(n)]
    free = [int(x) for x in v[3 + 3 * n:3 + 3 * n + nf]]
    return items, free, stop

  def _send_header(self, h: torch.Tensor) -> None:
    # headers go host-staged over the transport (a CUDA copy on RCCL): size first, then the body
    dev = self.dev
    self.t.isend(torch.tensor([float(h.numel())], dtype=torch.float64, device=dev), self.next)
    self.t.isend(h.to(dev), self.next)

  def _recv_header(self) -> torch.Tensor:
    dev = self.dev
    n = torch.empty(1, dtype=torch.float64, device=dev)
    self.t.recv(n, self.prev)
    h = torch.empty(int(n.item()), dtype=torch.float64, device=dev)
    self.t.recv(h, self.prev)
    return h.cpu()

  # ------------------------------------------------------------------ one lane step on this rank
  def _stage(self, items, x0: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
    """Run this rank's layers for a lane step; the last rank returns the sampled ids [B] int32 (device)."""
    rids = [str(k) for k, _, _ in items]
    qlens = [q for _, q, _ in items]
    if self.first:
      x = x0.to(self.dev)
    else:
      x = torch.empty(sum(qlens), self.D, dtype=torch.bfloat16, device=self.dev)
      self.t.wait(self.t.irecv(x, self.prev))
    y = self.r.forward(rids, qlens, x)
    if not self.last:
      self.t.isend(y.clone(), self.next)  # y may be a decode graph's static buffer
      return None
    temps = torch.tensor([t for _, _, t in items], dtype=torch.float32)
    if self.dev.type == "cuda":  # pinned + async: a pageable copy would wait here for the forward to finish
      temps = temps.pin_memory()
    temps = temps.to(self.dev, non_blocking=True)
    tok = K.sample(y, temps, self.top_k, self.seed_off)
    self.seed_off[1] += 1
    if self.world > 1:
      self.t.isend(tok, 0)
    return tok

  def _apply_free(self, free: List[int]) -> None:
    for k in free:
      self.r.free(str(k))

  # ------------------------------------------------------------------ rank 0: scheduler + first stage
  def _admit(self) -> None:
    room = self.max_batch - len(self._running)
    while room > 0:
      try:
        req = self._inbox.get_nowait()
      except queue.Empty:
        return
      req.key = self._next_key
      self._next_key += 1
      if not self.r.can_admit(str(req.key), len(req.ids) + req.max_tokens):
        self._emit(req.rid, [], True)  # cannot fit its context on this shard: finish it empty
        continue
      loads = [0] * self.lanes
      for q in self._running.values():
        loads[q.lane] += 1
      req.lane = loads.index(min(loads))
      self._running[req.rid] = req
      self._by_key[req.key] = req
      room -= 1

  def _collect(self, lane: int) -> None:
    """Rank 0: the ids of this lane's step in flight (the oldest step in flight: lanes run in a cycle)."""
    step = self._inflight[lane]
    if step is None:
      return
    self._inflight[lane] = None
    reqs, tok = step
    if tok is None:  # sampled on another rank
      tok = torch.empty(len(reqs), dtype=torch.int32, device=self.dev)
      self.t.wait(self.t.irecv(tok, self.world - 1))
    for req, t in zip(reqs, tok.tolist()):
      req.out.append(int(t))
      fin = t in self.eos or len(req.out) >= req.max_tokens
      self._emit(req.rid, [int(t)], fin)
      if fin:
        del self._running[req.rid]
        del self._by_key[req.key]
        self.r.free(str(req.key))
        self._free.append(req.key)

  def _launch(self, lane: int, stop: bool = False) -> bool:
    """Rank 0: start this lane's next step (prompts admitted to it, then its decoding requests).
    Returns whether anything was sent."""
    reqs = [q for q in self._running.values() if q.lane == lane] if not stop else []
    if not reqs and not (stop or (self._free and self.world > 1 and self._idle_lanes())):
      return False
    items, ids = [], []
    for q in reqs:
      if q.out:
        items.append((q.key, 1, q.temp))
        ids.append(q.out[-1])
      else:
        items.append((q.key, len(q.ids), q.temp))
        ids += q.ids
    free, self._free = self._free, []
    if self.world > 1:
      self._send_header(self._header(items, free, stop))
    if items:
      tok = self._stage(items, torch.tensor(ids, dtype=torch.int32))
      self._inflight[lane] = (reqs, tok)
    return True

  def _idle_lanes(self) -> bool:
    return all(s is None for s in self._inflight)

  def serve_forever(self, idle_wait: float = 0.5) -> None:
    """Rank 0 cycles through the lanes: collect a lane's ids, admit, launch its next step.  Other ranks
    follow the headers.  Rank 0 waits up to idle_wait for work when nothing is running."""
    if self.rank != 0:
      self._follow()
      return
    lane = 0
    while True:
      self._collect(lane)
      if self._stop:
        if all(s is None for s in self._inflight):
          break
        lane = (lane + 1) % self.lanes
        continue
      self._admit()
      launched = self._launch(lane)
      if not launched and self.idle() and all(s is None for s in self._inflight):
        self._wake.wait(idle_wait)
        self._wake.clear()
      lane = (lane + 1) % self.lanes
    if self.world > 1:  # stop (with the last frees) travels the ring; followers exit on it
      free, self._free = self._free, []
      self._send_header(self._header([], free, True))
    self.t.drain()

  # ------------------------------------------------------------------ ranks 1..N-1
  def _follow(self) -> None:
    while True:
      h = self._recv_header()
      items, free, stop = self._parse(h)
      if not self.last:
        self._send_header(h)
      self._apply_free(free)
      if items:
        self._stage(items, None)
      if stop:
        break
    self.t.drain()


# ---------------------------------------------------------------------- API adapter + process spawner
class _Engine:
  """What the ChatGPT API reads from `node.inference_engine` (tokenizer, eos ids, shard)."""

  def __init__(self, shard, tokenizer, eos_ids):
    self.shard, self.tokenizer, self.eos_token_ids = shard, tokenizer, tuple(eos_ids)
    from ..download.shard_download import NoopShardDownloader
    self.shard_downloader = NoopShardDownloader()


class RingNode:
  """Node-shaped front for a RingServer on rank 0, so `api/chatgpt_api.py` serves the GPU ring unchanged:
  process_prompt -> tokenize + submit; server tokens -> on_token callbacks on the asyncio loop
  (reference contract: node.py:109-147 fires on_token(request_id, [token], is_finished))."""

  def __init__(self, server: RingServer, shard, tokenizer, eos_ids, default_temp: float, max_generate_tokens: int,
               loop=None, topology=None):
    from ..helpers import AsyncCallbackSystem
    self.srv = server
    self.inference_engine = _Engine(shard, tokenizer, eos_ids)
    self.default_temp, self.max_generate_tokens = default_temp, max_generate_tokens
    self.on_token = AsyncCallbackSystem()
    self.node_download_progress = {}
    self.current_topology = topology
    self.server = None
    self.loop = loop
    server.on_token(self._from_server)

  def _from_server(self, rid, toks, fin):
    if self.loop is not None:
      self.loop.call_soon_threadsafe(self.on_token.trigger_all, rid, list(toks), fin)
    else:
      self.on_token.trigger_all(rid, list(toks), fin)

  async def process_prompt(self, base_shard, prompt: str, request_id: Optional[str] = None, inference_state=None):
    st = inference_state or {}
    temp = st.get("temperature")
    mt = st.get("max_tokens") or self.max_generate_tokens
    ids = self.inference_engine.tokenizer.encode(prompt)
    self.srv.submit(request_id, ids, self.default_temp if temp is None else float(temp), int(mt))


def _serve_worker(rank: int, world: int, port: int, a: dict) -> None:
  import asyncio
  import os
  os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                    MASTER_PORT=str(port))
  from ..inference.shard import Shard
  from ..inference.tokenizers import _resolve_tokenizer
  from ..models import registry
  from ..models.config import load_config, preset
  from ..models.weights import load_hf_weights
  from ..runtime.runner import ShardRunner
  from ..topology.ring_memory_weighted_partitioning_strategy import equal_layer_shards
  from ..train.ring_train import _model_dir
  from .comm import P2PTransport, init_distributed

  rank, world, dev = init_distributed()
  ctl = dist.new_group(backend="gloo") if world > 1 else None
  model = a["model"]
  mdir = _model_dir(model)
  cfg = load_config(mdir) if mdir is not None else preset(model)
  shard = equal_layer_shards(model, cfg.num_layers, world)[rank]
  weights = load_hf_weights(mdir, cfg, shard, dev) if mdir is not None and any(mdir.glob("*.safetensors")) else None
  runner = ShardRunner(cfg, shard, dev, weights=weights, max_batch=a["max_batch"], max_ctx=a["max_ctx"], seed=0)
  srv = RingServer(runner, rank, world, P2PTransport(rank, world), ctl, eos_ids=cfg.eos_token_ids)
  print(f"[ring {rank}/{world}] {model} layers {shard.start_layer}-{shard.end_layer} on {dev}"
        + ("" if weights is not None else " (random-init weights: no local checkpoint)"), flush=True)
  if rank == 0:
    tok = _resolve_tokenizer(mdir if mdir is not None else (registry.get_repo(model, "ShardedInferenceEngine") or "byte"),
                             cfg.vocab_size)
    full = Shard(model, 0, cfg.num_layers - 1, cfg.num_layers)
    asyncio.run(_rank0_main(srv, full, tok, cfg, a))
  else:
    srv.serve_forever()
  if world > 1:
    dist.destroy_process_group()


async def _rank0_main(srv: RingServer, shard, tok, cfg, a: dict) -> None:
  import asyncio
  loop = asyncio.get_running_loop()
  node = RingNode(srv, shard, tok, cfg.eos_token_ids, a["default_temp"], a["max_generate_tokens"], loop=loop)
  th = threading.Thread(target=srv.serve_forever, name="xot-ring-rounds", daemon=True)
  th.start()
  try:
    if a.get("prompt") is not None:  # `xot run <model> --ring`: one prompt, print the answer
      done = asyncio.Event()
      out: List[int] = []

      def on_tok(rid, toks, fin):
        out.extend(toks)
        if fin:
          done.set()

      node.on_token.register("run").on_next(on_tok)
      await node.process_prompt(shard, a["prompt"], request_id="run-0",
                                inference_state={"max_tokens": a["max_generate_tokens"]})
      await asyncio.wait_for(done.wait(), timeout=600)
      print(tok.decode([t for t in out if t not in set(cfg.eos_token_ids)]), flush=True)
      return
    from ..api.chatgpt_api import ChatGPTAPI
    api = ChatGPTAPI(node, "ShardedInferenceEngine", response_timeout=a["response_timeout"],
                     default_model=a["model"], system_prompt=a.get("system_prompt"))
    await api.run(port=a["api_port"])
    print(f"[ring 0] ChatGPT API on :{a['api_port']} (RCCL ring of {srv.world})", flush=True)
    await asyncio.Event().wait()
  finally:
    srv.stop()
    await asyncio.get_running_loop().run_in_executor(None, th.join, 60)


def serve_ring(args) -> int:
  """`xot [run] <model> --ring --gpus N`: one process per GPU, continuous-batching ring over RCCL."""
  import os
  import torch.multiprocessing as mp
  from ..train.ring_train import _free_port
  n = args.gpus or max(1, torch.cuda.device_count())
  model = getattr(args, "model_name", None) or getattr(args, "run_model", None) or args.default_model
  a = {"model": model, "max_batch": int(os.environ.get("XOT_MAX_BATCH", 64)),
       "max_ctx": int(os.environ.get("XOT_MAX_CTX", 8192 if torch.cuda.is_available() else 2048)),
       "default_temp": args.default_temp, "max_generate_tokens": args.max_generate_tokens,
       "api_port": args.chatgpt_api_port, "response_timeout": args.chatgpt_api_response_timeout,
       "system_prompt": getattr(args, "system_prompt", None),
       "prompt": args.prompt if (args.command == "run" or getattr(args, "run_model", None)) else None}
  port = _free_port()
  if n == 1:
    _serve_worker(0, 1, port, a)
    return 0
  ctx = mp.get_context("spawn")
  procs = [ctx.Process(target=_serve_worker, args=(r, n, port, a)) for r in range(n)]
  for p in procs:
    p.start()
  rc = 0
  for p in procs:
    p.join()
    rc = rc or (p.exitcode or 0)
  return rc

"""Serving over the local GPU ring: continuous batching with the activation hand-off on RCCL.

The reference serves one request at a time, moving every hop through gRPC with the JSON state
(xotorch/orchestration/node.py:109-147, 403-443; grpc_peer_handle.py:117-136).  Here the GPUs of one
host are the ring peers (one process each) and the data plane is RCCL p2p over xGMI:

  control plane  rank 0 (API, tokenizer, scheduler) broadcasts one small message per round over a gloo
                 group: the requests admitted this round (rid, prompt ids), the order of the running
                 batch, and the requests to free.  Every rank therefore knows every tensor shape it
                 will receive, so the data plane carries bare activations: no headers, no state.
  data plane     per round: one prefill pass for the admitted prompts (if any), then one decode pass for
                 the running batch.  Stage r receives [T, D] bf16 from r-1, runs its layers, sends to
                 r+1; the last stage samples on device (temperature / top-k 35) and sends the ids [B]
                 int32 back to rank 0 (P2PTransport: one communicator per directed edge).
  KV             each rank holds the paged KV of its own layers for every running request; a finished
                 request is freed on every rank in the next round's message.

`RingServer.submit()` is thread-safe (the asyncio API calls it); tokens come back through `on_token`
callbacks (request_id, [token], is_finished) — the reference's token callback contract.
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


class RingServer:
  def __init__(self, runner, rank: int, world: int, transport, ctl_group=None, eos_ids: Sequence[int] = (),
               top_k: int = 35, seed: int = 1234, max_batch: Optional[int] = None):
    self.r, self.rank, self.world, self.t = runner, rank, world, transport
    self.ctl = ctl_group
    self.first, self.last = runner.shard.is_first_layer(), runner.shard.is_last_layer()
    self.prev, self.next = (rank - 1) % world, (rank + 1) % world
    self.D = runner.config.hidden_size
    self.eos = set(int(e) for e in eos_ids)
    self.top_k = top_k
    self.seed_off = torch.tensor([seed, 0], dtype=torch.int64, device=runner.device)
    self.max_batch = max_batch or runner.max_batch
    self._inbox: "queue.Queue[_Req]" = queue.Queue()
    self._running: Dict[str, _Req] = {}
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

  # ------------------------------------------------------------------ one round
  def _plan(self, free: List[str]) -> dict:
    """Rank 0: admit queued requests that fit, and fix this round's batch order."""
    new = []
    room = self.max_batch - len(self._running)
    while room > 0:
      try:
        req = self._inbox.get_nowait()
      except queue.Empty:
        break
      if not self.r.can_admit(req.rid, len(req.ids) + req.max_tokens):
        self._emit(req.rid, [], True)  # cannot fit its context on this shard: finish it empty
        continue
      new.append(req)
      room -= 1
    for req in new:
      self._running[req.rid] = req
    decode = [rid for rid in self._running if self._running[rid].out]
    return {"new": [(q.rid, q.ids, q.temp) for q in new], "decode": decode,
            "temps": [self._running[r].temp for r in decode], "free": list(free), "stop": self._stop}

  def _broadcast(self, msg: Optional[dict]) -> dict:
    if self.world == 1:
      return msg
    box = [msg]
    dist.broadcast_object_list(box, src=0, group=self.ctl)
    return box[0]

  def _pass(self, groups) -> Optional[List[List[int]]]:
    """One pipeline pass of a round's micro-batches through this rank.  groups: [(rids, qlens, x0, temps)].
    Micro-batch m+1 enters this stage while m is on the next one (sends are async), so with M >= world
    micro-batches every GPU of the ring works at once.  Returns the sampled ids per group on rank 0."""
    dev = self.r.device
    local = []
    for rids, qlens, x0, temps in groups:
      if self.first:
        x = x0
      else:
        x = torch.empty(sum(qlens), self.D, dtype=torch.bfloat16, device=dev)
        self.t.wait(self.t.irecv(x, self.prev))
      y = self.r.forward(rids, qlens, x)
      if not self.last:
        self.t.isend(y.clone(), self.next)  # y may be a decode graph's static buffer
        continue
      tok = K.sample(y, temps.to(dev), self.top_k, self.seed_off)
      self.seed_off[1] += 1
      if self.world > 1:
        self.t.isend(tok, 0)
      local.append(tok)
    if self.rank != 0:
      return None
    res = []
    for g, (rids, _, _, _) in enumerate(groups):
      if self.last:
        tok = local[g]
      else:
        tok = torch.empty(len(rids), dtype=torch.int32, device=dev)
        self.t.wait(self.t.irecv(tok, self.world - 1))
      res.append(tok.tolist())
    return res

  def _emit(self, rid: str, toks: List[int], fin: bool) -> None:
    for cb in self._callbacks:
      cb(rid, toks, fin)

  def _collect(self, rids: List[str], toks: List[int], free: List[str]) -> None:
    for rid, t in zip(rids, toks):
      req = self._running[rid]
      req.out.append(t)
      fin = t in self.eos or len(req.out) >= req.max_tokens
      self._emit(rid, [t], fin)
      if fin:
        del self._running[rid]
        free.append(rid)

  def step(self, free: List[str]) -> bool:
    """One round on every rank (rank 0 plans; the others follow its message).  Returns False at stop."""
    msg = self._broadcast(self._plan(free) if self.rank == 0 else None)
    for rid in msg["free"]:
      if self.r.has(rid):
        self.r.free(rid)
    free.clear()
    if msg["new"]:
      rids = [rid for rid, _, _ in msg["new"]]
      lens = [len(ids) for _, ids, _ in msg["new"]]
      x0 = torch.tensor([i for _, ids, _ in msg["new"] for i in ids], dtype=torch.int32) if self.first else None
      temps = torch.tensor([t for _, _, t in msg["new"]], dtype=torch.float32)
      toks = self._pass([(rids, lens, x0, temps)])
      if self.rank == 0:
        self._collect(rids, toks[0], free)
    if msg["decode"]:
      rids, temps = msg["decode"], msg["temps"]
      M = min(self.world, len(rids))  # micro-batches in flight: one per stage fills the ring
      per = -(-len(rids) // M)
      groups = []
      for lo in range(0, len(rids), per):
        g = rids[lo:lo + per]
        x0 = torch.tensor([self._running[r].out[-1] for r in g], dtype=torch.int32) if self.first else None
        groups.append((g, [1] * len(g), x0, torch.tensor(temps[lo:lo + per], dtype=torch.float32)))
      toks = self._pass(groups)
      if self.rank == 0:
        for (g, _, _, _), tk in zip(groups, toks):
          self._collect(g, tk, free)
    return not msg["stop"]

  def serve_forever(self, idle_wait: float = 0.5) -> None:
    """Round loop (every rank).  Rank 0 waits up to idle_wait for work when nothing is running, then
    runs a round anyway (an empty message keeps the followers' control-plane waits short)."""
    free: List[str] = []
    while True:
      if self.rank == 0 and self.idle() and not free and not self._stop:
        self._wake.wait(idle_wait)
        self._wake.clear()
      if not self.step(free):
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

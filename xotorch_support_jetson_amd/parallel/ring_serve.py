"""Serving over the local GPU ring: continuous batching with the activation hand-off on RCCL.

The reference serves one request at a time, moving every hop through gRPC with the JSON state
(xotorch/orchestration/node.py:109-147, 403-443; grpc_peer_handle.py:117-136).  Here the GPUs of one
host are the ring peers (one process each, `xot --gpus N`) and the data plane is RCCL p2p over xGMI.

  lanes          rank 0 (API, tokenizer, scheduler) splits the running requests into `world` lanes (times
                 XOT_RING_LANES_PER_RANK) and
                 cycles through them: a lane's next step starts as soon as its previous step's tokens are
                 back, while the other lanes' steps are on the other GPUs -- the ring stays full, as in
                 bench.py, instead of filling and draining once per round.
  control plane  each lane step is announced ahead of its data by a fixed-size header (float64: the step's
                 requests as (wire id, new tokens, temperature), requests to free, a stop flag) sent over a
                 gloo group, i.e. host to host: a follower reads it without touching its GPU stream, so it
                 queues the step's receive + forward while its previous step is still running (a header on
                 the RCCL stream would be readable only after that stream drained).
  data plane     stage r receives [T, D] bf16 from r-1, runs its layers, sends to r+1 (P2PTransport: one
                 communicator per directed edge).  The ring ends share the LM head as in bench.py
                 (pipeline.RingStage, the same hand-off code): the last stage computes vocab rows [0, Vs) and
                 sends the normed hidden state + its top-k candidates to rank 0, which computes rows [Vs, V)
                 and samples on device (temperature / top-k 35); without the split the last stage samples and
                 sends the ids [B] int32.  Rank 0 receives lane steps' hand-offs in launch order (FIFO per edge).
  async steps    rank 0 never waits for a lane's ids before queueing that lane's next step: the running decoders
                 of the next step read their input ids straight from the device tensor the previous step
                 sampled, and the host reads those ids (tokens to emit, EOS) while the next step is already
                 on the GPU -- at world 1 the single lane keeps one step queued behind the running one.  A
                 request that turns out to have finished (EOS) had one speculative token computed: it is
                 discarded and the request's pages are freed as usual.
  prefill        prompts go through in chunks: a lane step carries at most `step_tokens` new tokens
                 (XOT_MAX_STEP_TOKENS), so a long prompt never stalls the other requests of its lane for a
                 whole-prompt forward; only the final chunk's sampled token is kept.
  KV             each rank holds the paged KV of its own layers for every running request.  All ranks size
                 their pools to the SMALLEST pool on the ring (min over ranks at start-up), so rank 0's
                 BlockManager -- which sees the same appends in the same order as every other rank's --
                 accounts for every rank exactly.  When a step would not fit, rank 0 preempts the youngest
                 requests of that lane: their pages are freed on every rank (the next header carries the
                 frees) and they are re-admitted later by re-prefilling prompt + tokens so far; their
                 streams continue where they stopped.  (Admission never rejects a request that fits
                 max_ctx; the old design refused any request whose whole budget did not fit at once.)
  failures       every rank runs a HealthMonitor (parallel/health.py: store heartbeats, communicator abort).
                 On a peer failure the survivors re-form a dense ring (reform_ring), re-partition the
                 layers over the live GPUs (memory-weighted, ring order), rebuild their shards, and rank 0
                 re-admits every running request with a re-prefill -- the reference re-partitions on the
                 next request after a peer drops (node.py:455-460, udp_discovery.py:204-246) but loses
                 the requests in flight.  The API owner (rank 0) itself cannot be replaced.

`RingServer.submit()` is thread-safe (the asyncio API calls it); tokens come back through `on_token`
callbacks (request_id, [token], is_finished) -- the reference's token callback contract.
"""
from __future__ import annotations

import collections
import os
import queue
import sys
import threading
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence

import torch
import torch.distributed as dist

from ..ops import kernels as K
from .health import FaultInjector, HealthMonitor, PeerFailure, reform_ring, wait_work

STEP_TOKENS = int(os.environ.get("XOT_MAX_STEP_TOKENS", "8192"))
OPS_CAP = 256  # KV operations per header (more go ahead of the step in op-only headers)
# prompt-prefix KV reuse on the ring (inference/prefix_cache.py policy on rank 0): at most this fraction of the pool
PREFIX_CACHE = os.environ.get("XOT_PREFIX_CACHE", "1") == "1"
PREFIX_CACHE_FRAC = float(os.environ.get("XOT_PREFIX_CACHE_FRAC", "0.25"))
# KV operations rank 0 performs on its BlockManager and every other rank repeats, in order, from the headers:
OP_FREE, OP_FREE_HOLDER, OP_FORK_TO_REQ, OP_FORK_TO_HOLDER = 1, 2, 3, 4  # (code, a, b, ntok)


class _RecordingBM:
  """Rank 0's BlockManager as the prefix cache sees it: holder forks and frees go through to the real one and
  are recorded as header operations, so every rank's pool changes the same way at the same point."""

  def __init__(self, bm, sink: list):
    self._bm, self._sink = bm, sink

  def __getattr__(self, name):
    return getattr(self._bm, name)

  @staticmethod
  def _holder_id(name: str) -> int:
    return int(name[3:]) if name.startswith("pc:") else -1

  def fork(self, src: str, dst: str, ntok: int) -> None:
    self._bm.fork(src, dst, ntok)
    h = self._holder_id(src)
    if h >= 0:
      self._sink.append((OP_FORK_TO_REQ, h, int(dst), ntok))
    else:
      self._sink.append((OP_FORK_TO_HOLDER, int(src), self._holder_id(dst), ntok))

  def free(self, name: str) -> None:
    self._bm.free(name)
    h = self._holder_id(name)
    self._sink.append((OP_FREE_HOLDER, h, 0, 0) if h >= 0 else (OP_FREE, int(name), 0, 0))


@dataclass
class _Req:
  rid: str
  ids: List[int]
  temp: float
  max_tokens: int
  out: List[int] = field(default_factory=list)
  key: int = -1  # integer id on the wire (a new one per admission)
  lane: int = -1
  fed: int = 0  # tokens of ids + out (+ pending samples) fed to the ring (in the KV cache or in a step in flight)
  pend: int = 0  # sampled tokens of steps in flight, not read on the host yet (0, 1, or 2 briefly)
  order: int = 0  # admission order: the largest is the youngest
  pixels: Optional[torch.Tensor] = None  # LLaVA: preprocessed images of the prompt (rank 0 = first shard)
  feats: Optional[torch.Tensor] = None  # their projected features [image tokens, D] (computed on first use)

  def todo(self) -> int:
    """Tokens still to feed before the next sampled token is a real output (1 while decoding)."""
    return len(self.ids) + len(self.out) + self.pend - self.fed

  def on_device(self) -> bool:
    """Its next token to feed is a sample still on the device (the lane's step in flight drew it)."""
    return self.pend > 0 and self.fed >= len(self.ids) + len(self.out)


class RingServer:
  def __init__(self, runner, rank: int, world: int, transport, ctl_group=None, eos_ids: Sequence[int] = (),
               top_k: int = 35, seed: int = 1234, max_batch: Optional[int] = None, step_tokens: Optional[int] = None,
               monitor: Optional[HealthMonitor] = None, make_runner: Optional[Callable] = None,
               pool_pages: Optional[int] = None, ops_cap: int = OPS_CAP, prefix_cache: Optional[bool] = None,
               lanes_per_rank: Optional[int] = None, split_head: Optional[bool] = None):
    self.r, self.rank, self.world, self.t = runner, rank, world, transport
    self.want_split = split_head
    # lanes per ring rank (XOT_RING_LANES_PER_RANK): with more than one, rank 0 has another lane's step queued
    # while it turns one lane's ids around on the host (collect, plan, header), at smaller steps per lane
    self.lanes_per_rank = max(1, lanes_per_rank or int(os.environ.get("XOT_RING_LANES_PER_RANK", "1")))
    self.ops_cap = max(1, ops_cap)  # KV operations per header
    self.use_prefix_cache = PREFIX_CACHE if prefix_cache is None else prefix_cache
    self.ctl = ctl_group  # gloo group of the control plane (headers); None with world 1
    self.eos = set(int(e) for e in eos_ids)
    self.top_k = top_k
    self.seed = seed
    self.max_batch = max_batch or runner.max_batch
    self.step_tokens = max(1, step_tokens or STEP_TOKENS)
    self.monitor = monitor
    self.make_runner = make_runner  # (shard) -> ShardRunner: rebuilds this rank's shard after a re-partition
    self.generation = 0
    self.backend = dist.get_backend() if dist.is_initialized() else "gloo"
    self._set_topology(runner, rank, world, pool_pages)
    self._gather_peers()
    self._inbox: "queue.Queue[_Req]" = queue.Queue()
    self._waiting: "collections.deque[_Req]" = collections.deque()  # preempted (front) and new requests
    self._running: Dict[str, _Req] = {}
    self._next_key = 0
    self._next_order = 0
    self._ops_sink()  # KV operations for every other rank (carried by the next headers, in order)
    self._callbacks: List[Callable[[str, List[int], bool], None]] = []
    self._stop = False
    self._wake = threading.Event()
    self._pending_ctl: list = []
    self.stats = {"steps": 0, "preempted": 0, "chunks": 0, "recoveries": 0}

  def _set_topology(self, runner, rank: int, world: int, pool_pages: Optional[int]) -> None:
    self.r, self.rank, self.world = runner, rank, world
    self.first, self.last = runner.shard.is_first_layer(), runner.shard.is_last_layer()
    self.prev, self.next = (rank - 1) % world, (rank + 1) % world
    self.D = runner.config.hidden_size
    self.dev = runner.device
    self._make_stage(runner, rank, world)
    self.lanes = max(1, world) * self.lanes_per_rank
    self._inflight: List[Optional[dict]] = [None] * self.lanes  # per lane: its step in flight (see _launch)
    # rank 0 plans with the smallest pool of the ring (exact for every rank: same appends everywhere)
    self.pool_pages = min(pool_pages or runner.bm.num_blocks, runner.bm.num_blocks)
    self.hcap = 4 + 3 * self.max_batch + 4 * self.ops_cap
    # rank 0 owns the prefix-cache policy; it runs on a recording view of its pool (every fork / free of a
    # holder becomes a header operation).  Headers reach every rank in order, so unlike the gRPC ring no
    # confirmation protocol is needed: an operation is applied everywhere before any step that depends on it.
    self.pc = None
    longrope = (runner.config.rope_scaling or {}).get("rope_type") == "longrope"
    if rank == 0 and self.use_prefix_cache and not longrope:
      from ..inference.prefix_cache import PrefixCache
      self.pc = PrefixCache(_RecordingBM(runner.bm, self._ops_sink()), int(self.pool_pages * PREFIX_CACHE_FRAC),
                            single_shard=True)

  def _make_stage(self, runner, rank: int, world: int) -> None:
    """The ring-stage helper shared with bench.py (pipeline.RingStage): sampler + seed, and at world > 1 the LM
    head split between the ring ends.  Every rank must take the same split decision: the first stage cannot
    derive its head rows for externally loaded weights without a head, so the flags are reduced (MIN) over the
    control group and every rank falls back to the unsplit head together."""
    from .pipeline import RingStage
    want = (os.environ.get("XOT_SPLIT_HEAD", "1") == "1") if self.want_split is None else self.want_split
    try:
      st = RingStage(runner, rank, world, self.t, top_k=self.top_k, seed=self.seed, split_head=want)
      ok = 1
    except ValueError:
      st, ok = None, 0
    if world > 1 and self.ctl is not None and want:
      flag = torch.tensor([ok], dtype=torch.int64)
      dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=self.ctl)
      ok = int(flag[0])
    if st is None or (st.split and not ok):
      runner.model.head_rows = None
      st = RingStage(runner, rank, world, self.t, top_k=self.top_k, seed=self.seed, split_head=False)
    self.ring = st
    self.seed_off = st.seed_off

  def _ops_sink(self) -> list:
    if not hasattr(self, "_ops"):
      self._ops = []
    return self._ops

  def _gather_peers(self) -> None:
    """Collective over the control group (every rank, at start-up and after a re-form): each rank's device
    capabilities and layer range.  Rank 0 keeps them as the orchestration layer's Topology -- one peer per
    GPU, ring edges labelled with the data plane -- and the ring's partitions, so /v1/topology, tinychat's
    topology panel and the TUI show the GPU ring like the reference shows its discovered peers
    (orchestration/node.py:533-566)."""
    import socket
    from ..topology.device_capabilities import DeviceCapabilities, device_capabilities
    from ..topology.partitioning_strategy import Partition
    from ..topology.topology import Topology
    dev = self.r.device
    local = dev.index if dev.type == "cuda" and dev.index is not None else self.rank
    mine = {"id": f"{socket.gethostname()}-gpu{local}", "caps": device_capabilities(local_gpu=local).model_dump(),
            "layers": (self.r.shard.start_layer, self.r.shard.end_layer)}
    peers = [mine]
    if self.world > 1 and self.ctl is not None:
      peers = [None] * self.world
      dist.all_gather_object(peers, mine, group=self.ctl)
    ids = [p["id"] for p in peers]
    if len(set(ids)) != len(ids):  # e.g. CPU ranks of one host: fall back to ring positions
      ids = [f"{p['id']}-r{i}" for i, p in enumerate(peers)]
    self.node_ids = ids
    link = "xGMI (RCCL p2p)" if self.backend == "nccl" else f"{self.backend} p2p"
    t = Topology()
    for nid, p in zip(ids, peers):
      t.update_node(nid, DeviceCapabilities(**p["caps"]))
    for i in range(self.world if self.world > 1 else 0):
      t.add_edge(ids[i], ids[(i + 1) % self.world], link)
    t.active_node_id = ids[0]
    L = self.r.shard.n_layers
    self.topology = t
    self.partitions = [Partition(nid, p["layers"][0] / L, (p["layers"][1] + 1) / L) for nid, p in zip(ids, peers)]
    self.layer_ranges = [(nid, p["layers"][0], p["layers"][1]) for nid, p in zip(ids, peers)]

  # ------------------------------------------------------------------ rank-0 API side
  def submit(self, rid: str, ids: Sequence[int], temp: float = 0.0, max_tokens: int = 256,
             pixels: Optional[torch.Tensor] = None) -> None:
    """pixels: [N, 3, S, S] images whose image-token runs the ids carry (LLaVA; models/vision.py)."""
    self._inbox.put(_Req(rid, [int(i) for i in ids], float(temp), int(max_tokens), pixels=pixels))
    self._wake.set()

  def on_token(self, cb: Callable[[str, List[int], bool], None]) -> None:
    self._callbacks.append(cb)

  def stop(self) -> None:
    self._stop = True
    self._wake.set()

  def idle(self) -> bool:
    return not self._running and not self._waiting and self._inbox.empty()

  def _emit(self, rid: str, toks: List[int], fin: bool) -> None:
    for cb in self._callbacks:
      cb(rid, toks, fin)

  # ------------------------------------------------------------------ control plane (gloo, host to host)
  def _header(self, items, ops, stop: bool) -> torch.Tensor:
    """[n_items, n_ops, stop, generation, (key, qlen, temp) * n_items, (code, a, b, ntok) * n_ops, 0 ...]
    float64 of fixed size hcap (exact for ids < 2^53).  The ops (KV frees and prefix-cache forks) are applied
    before the step's forward, in order."""
    h = torch.zeros(self.hcap, dtype=torch.float64)
    vals = [float(len(items)), float(len(ops)), 1.0 if stop else 0.0, float(self.generation)]
    for key, qlen, temp in items:
      vals += [float(key), float(qlen), float(temp)]
    for op in ops:
      vals += [float(x) for x in op]
    h[:len(vals)] = torch.tensor(vals, dtype=torch.float64)
    return h

  @staticmethod
  def _parse(h: torch.Tensor):
    v = h.tolist()
    n, no, stop = int(v[0]), int(v[1]), v[2] != 0.0
    items = [(int(v[4 + 3 * i]), int(v[5 + 3 * i]), v[6 + 3 * i]) for i in range(n)]
    o = 4 + 3 * n
    ops = [tuple(int(x) for x in v[o + 4 * i:o + 4 * i + 4]) for i in range(no)]
    return items, ops, stop

  def _send_header(self, h: torch.Tensor) -> None:
    if self.monitor is not None:
      self.monitor.check()
    self._pending_ctl.append((dist.isend(h, self.next, group=self.ctl), h))
    self._pending_ctl = [(w, t) for w, t in self._pending_ctl if not w.is_completed()]

  def _recv_header(self) -> torch.Tensor:
    h = torch.empty(self.hcap, dtype=torch.float64)
    wait_work(dist.irecv(h, self.prev, group=self.ctl), self.monitor)
    return h

  # ------------------------------------------------------------------ one lane step on this rank
  def _stage(self, items, x0: Optional[torch.Tensor], image_embeds: Optional[torch.Tensor] = None,
             gather=None, temps: Optional[torch.Tensor] = None) -> Optional[torch.Tensor]:
    """Run this rank's layers for a lane step.  Rank 0's input ids are x0 (host) with the rows `gather` =
    (rows in x, device ids of the previous step, rows there) filled on the device.  The last rank samples (or,
    with the split head, sends its head share to rank 0); returns the sampled ids [B] int32 (device) where
    they are drawn on this rank, else None."""
    rids = [str(k) for k, _, _ in items]
    qlens = [q for _, q, _ in items]
    if self.first:
      if self.dev.type == "cuda":  # pinned + async: a pageable copy would wait for everything queued before it
        x0 = x0.pin_memory()
      x = x0.to(self.dev, non_blocking=True)
      if gather is not None:
        at, prev, rows = gather
        x.index_copy_(0, at, prev.index_select(0, rows))
    else:
      x = torch.empty(sum(qlens), self.D, dtype=torch.bfloat16, device=self.dev)
      self.t.wait(self.t.irecv(x, self.prev))
    y = (self.r.forward(rids, qlens, x) if image_embeds is None
         else self.r.forward(rids, qlens, x, image_embeds=image_embeds))
    if not self.last:
      self.t.isend(y.clone(), self.next)  # y may be a decode graph's static buffer
      return None
    if self.ring.split:  # the last stage's share of the head + its top-k candidates -> rank 0
      self.ring._send_item(self.ring._head_part(y))
      return None
    if temps is None:
      temps = self._temps(items)
    tok = self.ring._sample(y, temps)
    if self.world > 1:
      self.t.isend(tok, 0)
    return tok

  def _temps(self, items) -> torch.Tensor:
    temps = torch.tensor([t for _, _, t in items], dtype=torch.float32)
    if self.dev.type == "cuda":  # pinned + async: a pageable copy would wait here for the queued work
      temps = temps.pin_memory()
    return temps.to(self.dev, non_blocking=True)

  def _resolve(self, step: dict) -> torch.Tensor:
    """Rank 0: the device ids of its oldest step in flight.  At world 1 they were sampled by _stage; otherwise
    the last stage's hand-off is received (a stream dependency, no host wait) and, with the split head, the
    remaining head rows + the sampler run here.  Called in launch order (the hand-offs arrive FIFO)."""
    if step["tok"] is None:
      B = len(step["plan"])
      if self.ring.split:
        step["tok"] = self.ring._finish_head(*self.ring._recv_item(B), step["temps"])
      else:
        tok = torch.empty(B, dtype=torch.int32, device=self.dev)
        self.t.wait(self.t.irecv(tok, self.world - 1))
        step["tok"] = tok
    return step["tok"]

  def _apply_ops(self, ops) -> None:
    """Followers: repeat rank 0's KV operations on this rank's pool (same order, same point in the steps)."""
    from ..inference.prefix_cache import holder
    bm = self.r.bm
    for code, a, b, ntok in ops:
      if code == OP_FREE:
        self.r.free(str(a))
      elif code == OP_FREE_HOLDER:
        bm.free(holder(a))
      elif code == OP_FORK_TO_REQ:
        bm.fork(holder(a), str(b), ntok)
      elif code == OP_FORK_TO_HOLDER:
        bm.fork(str(a), holder(b), ntok)

  # ------------------------------------------------------------------ rank 0: scheduler + first stage
  def _free_pages(self) -> int:
    bm = self.r.bm
    return bm.num_free - (bm.num_blocks - self.pool_pages)

  def _pages(self, q: _Req, n: int) -> int:
    return self.r.bm.blocks_needed(str(q.key), n) if self.r.has(str(q.key)) else -(-n // 64)

  def _release(self, q: _Req) -> None:
    """Drop a request's pages here and (via the next headers) on every other rank."""
    if self.r.has(str(q.key)):
      self.r.free(str(q.key))
    self._ops.append((OP_FREE, q.key, 0, 0))
    if self.pc is not None:
      self.pc.on_finish(str(q.key))

  def _admit(self) -> None:
    while True:
      try:
        self._waiting.append(self._inbox.get_nowait())
      except queue.Empty:
        break
    reserve = sum(1 for q in self._running.values() if q.todo() <= 1)  # one page of growth per decoder
    while self._waiting and len(self._running) < self.max_batch:
      q = self._waiting[0]
      total = len(q.ids) + len(q.out)
      if total + 1 > self.r.max_ctx or -(-(total + 1) // 64) > self.pool_pages:
        self._waiting.popleft()  # can never fit on this ring: finish it (length)
        self._emit(q.rid, [], True)
        continue
      first = min(total, self.step_tokens)
      if self._running and self._free_pages() - -(-first // 64) < reserve:
        break  # wait for pages (an empty ring always admits: preemption makes the room)
      self._waiting.popleft()
      q.key, self._next_key = self._next_key, self._next_key + 1
      q.order, self._next_order = self._next_order, self._next_order + 1
      q.fed = 0
      loads = [0] * self.lanes
      for o in self._running.values():
        loads[o.lane] += 1
      q.lane = loads.index(min(loads))
      self._running[q.rid] = q
      reserve += 1

  def _preempt(self, q: _Req) -> None:
    self._release(q)
    del self._running[q.rid]
    q.lane, q.fed, q.pend = -1, 0, 0  # a sample still in flight is dropped (re-prefill resumes from q.out)
    self._waiting.appendleft(q)
    self.stats["preempted"] += 1

  def _finishes(self, q: _Req) -> bool:
    """Known to finish once its pending samples are read (token budget or context), whatever they are."""
    return q.pend > 0 and (len(q.out) + q.pend >= q.max_tokens or len(q.ids) + len(q.out) + q.pend + 1 > self.r.max_ctx)

  def _plan(self, lane: int):
    """(req, new tokens) of this lane's next step: decoders first, then prompt chunks in admission order
    within the step's token budget; the youngest are preempted while the step's pages do not fit.  Requests
    certain to finish with the samples in flight get no further step."""
    reqs = sorted((q for q in self._running.values() if q.lane == lane and not self._finishes(q)),
                  key=lambda q: (q.todo() > 1, q.order))
    if self.pc is not None:  # new prompts: fork the longest cached prefix (whole pages) and feed only the rest
      for q in reqs:
        if q.fed == 0 and q.pixels is None and q.todo() > 1 and not self.r.has(str(q.key)):
          n, _ = self.pc.on_prompt(str(q.key), q.ids + q.out)
          q.fed = n
    while True:
      plan, budget = [], self.step_tokens
      for q in reqs:
        n = q.todo()
        if n > 1:
          n = min(n, budget)
        if n <= 0 or budget <= 0:
          continue
        budget -= n
        plan.append((q, n))
      need = sum(self._pages(q, n) for q, n in plan)
      if need <= self._free_pages() or not plan:
        return plan
      if self.pc is not None and self.pc.cached_pages():  # cached prefixes go before running requests
        self.pc.evict(need + (self.r.bm.num_blocks - self.pool_pages))
        if need <= self._free_pages():
          return plan
      victim = max(reqs, key=lambda q: q.order)
      reqs.remove(victim)
      self._preempt(victim)

  def _collect(self, step: dict) -> None:
    """Rank 0: read a step's ids on the host (the next step of its lane is already queued behind it) and emit
    the real outputs; finished requests are released (a speculative token of theirs in the next step is
    ignored when that step is collected: the request is gone or re-admitted under another key)."""
    toks = self._resolve(step).tolist()
    if self.monitor is not None:
      self.monitor.check()  # an aborted transfer delivers garbage: never emit it
    for (q, n, real, key), t in zip(step["plan"], toks):
      if not real or self._running.get(q.rid) is not q or q.key != key:
        continue
      q.pend -= 1
      q.out.append(int(t))
      fin = (t in self.eos or len(q.out) >= q.max_tokens or len(q.ids) + len(q.out) + 1 > self.r.max_ctx)
      self._emit(q.rid, [int(t)], fin)
      if fin:
        del self._running[q.rid]
        self._release(q)

  def _launch(self, lane: int, prev: Optional[dict] = None, stop: bool = False) -> Optional[dict]:
    """Rank 0: start this lane's next step.  `prev` is the lane's step still in flight: decoders whose next
    input is a sample of it read that id from its device tensor.  Returns the step (None if nothing ran):
    {plan: [(req, n, real, key)], tok: device ids or None until _resolve, temps}."""
    plan = self._plan(lane) if not stop else []
    if not plan and not (stop or (self._ops and self.world > 1 and self._idle_lanes())):
      return None
    items, ids, embeds, steps = [], [], [], []
    at, rows = [], []
    for q, n in plan:
      items.append((q.key, n, q.temp))
      real = q.todo() == n  # this chunk completes what is known: its sample is the next output
      if q.on_device():
        assert n == 1 and prev is not None, "a pending sample without its step"
        at.append(len(ids))
        rows.append(prev["row"][q.key])
        ids.append(0)
      else:
        seq = q.ids + q.out
        ids += seq[q.fed:q.fed + n]
      if n > 1:
        self.stats["chunks"] += 1
      if q.pixels is not None:
        e = self._image_rows(q, q.ids + q.out, n)
        if e is not None:
          embeds.append(e)
      elif self.pc is not None and n == 1 and q.todo() == 1:
        self.pc.on_decode(str(q.key))  # its first decode step: keep the prompt's pages as a cached prefix
      steps.append((q, n, real, q.key))
    # Rank 0 has already applied these operations (frees, prefix forks) and planned this step on top of
    # them: every one must reach the other ranks AHEAD of the step (headers arrive in order), so operations
    # beyond one header's cap go first in op-only headers.
    ops = self._flush_ops()
    if self.world > 1:
      self._send_header(self._header(items, ops, stop))
    if not items:
      return None
    gather = None
    if at:
      pin = self.dev.type == "cuda"
      mk = (lambda v: torch.tensor(v, dtype=torch.int64).pin_memory().to(self.dev, non_blocking=True)) if pin else \
          (lambda v: torch.tensor(v, dtype=torch.int64))
      gather = (mk(at), self._resolve(prev), mk(rows))
    temps = self._temps(items)
    tok = self._stage(items, torch.tensor(ids, dtype=torch.int32), torch.cat(embeds) if embeds else None,
                      gather=gather, temps=temps)
    for q, n, real, _ in steps:
      q.fed += n
      if real:
        q.pend += 1
    self.stats["steps"] += 1
    return {"plan": steps, "tok": tok, "temps": temps, "row": {key: i for i, (_, _, _, key) in enumerate(steps)}}

  def _image_rows(self, q: _Req, seq: List[int], n: int) -> Optional[torch.Tensor]:
    """Rank 0 (first shard): the projected image features of the image tokens in this step's chunk
    seq[fed:fed + n] of an image prompt, in token order (the features replace those rows)."""
    img = self.r.config.image_token_id
    before = sum(1 for t in seq[:q.fed] if t == img)
    k = sum(1 for t in seq[q.fed:q.fed + n] if t == img)
    if not k:
      return None
    if q.feats is None:
      q.feats = self.r.image_features(q.pixels)
    return q.feats[before:before + k]

  def _flush_ops(self) -> List[tuple]:
    """Send op-only headers until at most ops_cap operations are pending; return (and clear) those."""
    if self.world > 1:
      while len(self._ops) > self.ops_cap:
        self._send_header(self._header([], self._ops[:self.ops_cap], False))
        del self._ops[:self.ops_cap]
    ops = list(self._ops)
    self._ops.clear()  # the prefix cache's recording view appends to this same list
    return ops

  def _idle_lanes(self) -> bool:
    return all(s is None for s in self._inflight)

  def serve_forever(self, idle_wait: float = 0.5) -> None:
    """Rank 0 cycles through the lanes: collect a lane's ids, admit, launch its next step.  Other ranks
    follow the headers.  Rank 0 waits up to idle_wait for work when nothing is running.  A peer failure
    re-forms the ring over the survivors and serving continues (see the module docstring)."""
    while True:
      try:
        if self.rank != 0:
          self._follow()
        else:
          self._lead(idle_wait)
        return
      except PeerFailure as e:
        self._recover(e.dead)
      except RuntimeError:
        # a send / recv on a dead peer's connection can fail before the heartbeat has declared the peer
        # dead: give the monitor its detection window before treating the error as fatal
        m = self.monitor
        if m is None or not m.failed.wait(timeout=m.timeout + 4 * m.interval):
          raise
        self._recover(m.dead)

  def _lead(self, idle_wait: float) -> None:
    """Per lane: the step in flight gets its device ids (_resolve), the lane's next step is launched on top of
    them, and only then are the previous step's ids read on the host (_collect) -- so the GPU always has the
    lane's next step queued while the host emits tokens, plans and builds headers."""
    lane = 0
    while True:
      prev = self._inflight[lane]
      self._inflight[lane] = None
      nxt = None
      if not self._stop:
        if prev is not None:
          self._resolve(prev)
        self._admit()
        nxt = self._launch(lane, prev)
      if prev is not None:
        self._collect(prev)
      self._inflight[lane] = nxt
      if self._stop and all(s is None for s in self._inflight):
        break
      if nxt is None and prev is None and self.idle() and all(s is None for s in self._inflight):
        self._wake.wait(idle_wait)
        self._wake.clear()
      lane = (lane + 1) % self.lanes
    if self.world > 1:  # stop (with the last operations) travels the ring; followers exit on it
      self._send_header(self._header([], self._flush_ops(), True))
    self.t.drain()
    self._drain_ctl()
    if self.monitor is not None:
      self.monitor.stop()

  # ------------------------------------------------------------------ ranks 1..N-1
  def _follow(self) -> None:
    while True:
      h = self._recv_header()
      items, ops, stop = self._parse(h)
      if not self.last:
        self._send_header(h)
      self._apply_ops(ops)
      if items:
        self._stage(items, None)
      if stop:
        break
    self.t.drain()
    self._drain_ctl()
    if self.monitor is not None:
      self.monitor.stop()

  def _drain_ctl(self) -> None:
    for w, _ in self._pending_ctl:
      try:
        w.wait()
      except Exception:
        pass
    self._pending_ctl = []

  # ------------------------------------------------------------------ failure recovery
  def _recover(self, dead: Sequence[int]) -> None:
    """Survivors: re-form a dense ring, re-partition the layers over it, rebuild this rank's shard; rank 0
    re-admits every running request (re-prefill of prompt + tokens so far)."""
    alive = [r for r in range(self.world) if r not in set(dead)]
    if 0 not in alive or self.make_runner is None or self.rank not in alive:
      raise PeerFailure(dead, "the API rank is gone or this server cannot rebuild its shard")
    if self.monitor is not None:
      self.monitor.stop()  # it would otherwise keep watching the old ring and abort the new groups
    self.generation += 1
    self.stats["recoveries"] += 1
    print(f"[ring {self.rank}] peer(s) {sorted(dead)} failed: re-forming the ring over {alive} "
          f"(generation {self.generation})", flush=True)
    self._pending_ctl = []
    new_rank, new_world = reform_ring(alive, self.rank, self.generation, backend=self.backend)
    from .comm import P2PTransport
    ctl = control_group() if new_world > 1 else None
    monitor = None
    if self.monitor is not None:
      monitor = HealthMonitor(new_rank, new_world, interval=self.monitor.interval, timeout=self.monitor.timeout,
                              generation=self.generation).start()
    # the fault injector (tests) stays with the original rank numbering: none after a re-form
    transport = P2PTransport(new_rank, new_world, monitor=monitor, injector=FaultInjector("", new_rank))
    old = self.r
    self.r = None
    del old  # free this GPU's old shard before building the new one
    if torch.cuda.is_available():
      torch.cuda.empty_cache()
    runner, pool = self.make_runner(new_rank, new_world, ctl)
    self.ctl, self.t, self.monitor = ctl, transport, monitor
    self._set_topology(runner, new_rank, new_world, pool)
    self._gather_peers()
    if self.rank == 0:
      for q in sorted(self._running.values(), key=lambda q: q.order, reverse=True):
        q.lane, q.fed, q.pend, q.feats = -1, 0, 0, None
        self._waiting.appendleft(q)  # oldest ends up first
      self._running.clear()
      self._ops.clear()  # the new shards start from empty pools (and a fresh prefix cache)


# ---------------------------------------------------------------------- API adapter + process spawner
class _Engine:
  """What the ChatGPT API and /metrics read from `node.inference_engine` (tokenizer, eos ids, shard, and rank
  0's runner: its KV pool mirrors every rank's, so its gauges are the ring's)."""

  def __init__(self, shard, tokenizer, eos_ids, server: Optional[RingServer] = None):
    self.shard, self.tokenizer, self.eos_token_ids = shard, tokenizer, tuple(eos_ids)
    self.srv = server
    from ..download.shard_download import NoopShardDownloader
    self.shard_downloader = NoopShardDownloader()

  @property
  def runner(self):
    return self.srv.r if self.srv is not None else None

  @property
  def prefix_cache(self):
    return self.srv.pc if self.srv is not None else None


class RingNode:
  """Node-shaped front for a RingServer on rank 0, so `api/chatgpt_api.py` serves the GPU ring unchanged:
  process_prompt -> tokenize + submit; server tokens -> on_token callbacks on the asyncio loop
  (reference contract: node.py:109-147 fires on_token(request_id, [token], is_finished))."""

  def __init__(self, server: RingServer, shard, tokenizer, eos_ids, default_temp: float, max_generate_tokens: int,
               loop=None, topology=None, config=None):
    from ..helpers import AsyncCallbackSystem
    self.srv = server
    self.inference_engine = _Engine(shard, tokenizer, eos_ids, server)
    self.config = config if config is not None else server.r.config
    self.default_temp, self.max_generate_tokens = default_temp, max_generate_tokens
    self.on_token = AsyncCallbackSystem()
    self.node_download_progress = {}
    self._topology = topology
    self.id = server.node_ids[0] if getattr(server, "node_ids", None) else "ring-0"
    self.server = None
    self.loop = loop
    server.on_token(self._from_server)

  @property
  def current_topology(self):
    """The ring's GPU peers (gathered by the server at start-up and after every re-form), for /v1/topology,
    tinychat and the TUI; an explicitly given topology wins."""
    return self._topology if self._topology is not None else getattr(self.srv, "topology", None)

  @property
  def partitions(self):
    return getattr(self.srv, "partitions", [])

  def layer_ranges(self):
    """[(peer id, first layer, last layer)] of the ring, in ring order."""
    return list(getattr(self.srv, "layer_ranges", []))

  def _from_server(self, rid, toks, fin):
    if self.loop is not None:
      self.loop.call_soon_threadsafe(self.on_token.trigger_all, rid, list(toks), fin)
    else:
      self.on_token.trigger_all(rid, list(toks), fin)

  async def process_prompt(self, base_shard, prompt: str, request_id: Optional[str] = None, inference_state=None):
    st = inference_state or {}
    temp = st.get("temperature")
    mt = st.get("max_tokens") or self.max_generate_tokens
    # `<|xot_image:URL|>` markers (the API keeps the chat's last image that way): a vision model's prompt gets
    # each image's token run and rank 0 -- the first shard -- splices the tower's features at prefill
    from ..models.vision import encode_with_images, image_pixels
    ids, urls = encode_with_images(self.inference_engine.tokenizer, self.config, prompt)
    pixels = None
    if urls:
      import asyncio
      pixels = await asyncio.get_running_loop().run_in_executor(None, image_pixels, self.config, urls)
    self.srv.submit(request_id, ids, self.default_temp if temp is None else float(temp), int(mt), pixels=pixels)


def control_group():
  """The gloo group that carries the headers: host to host, and with a week-long timeout (followers wait in
  a header receive for as long as the API has nothing to serve)."""
  import datetime
  return dist.new_group(backend="gloo", timeout=datetime.timedelta(days=7))


def ring_shards(model: str, num_layers: int, world: int, ctl=None):
  """Layer ranges of the ring's ranks, memory-weighted in ring order (every rank's total GPU memory,
  exchanged over the control group)."""
  from ..topology.ring_memory_weighted_partitioning_strategy import memory_weighted_layer_shards
  mem = 1
  if torch.cuda.is_available():
    mem = torch.cuda.get_device_properties(torch.cuda.current_device()).total_memory >> 20
  mems = [mem]
  if world > 1:
    t = torch.tensor([mem], dtype=torch.int64)
    out = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(out, t, group=ctl)
    mems = [int(x[0]) for x in out]
  return memory_weighted_layer_shards(model, num_layers, mems)


def min_pool_pages(runner, world: int, ctl=None) -> int:
  """The smallest KV pool (pages) of the ring: every rank sizes its plan to it."""
  n = torch.tensor([runner.bm.num_blocks], dtype=torch.int64)
  if world > 1:
    dist.all_reduce(n, op=dist.ReduceOp.MIN, group=ctl)
  return int(n[0])


def default_max_batch(cfg, world: int, avg_ctx: int = 512) -> int:
  """Running requests of the whole ring when XOT_MAX_BATCH is not set: as many as one rank's KV pool holds at
  `avg_ctx` tokens each (paged KV: requests grow on demand, preemption handles the rest), between 64 and 512
  per lane (512 = the batch where the decode GEMMs reach their tiles' rate, as in bench.py)."""
  if not torch.cuda.is_available():
    return 64
  from ..models.transformer import KVCache
  layers = -(-cfg.num_layers // world)
  total = torch.cuda.get_device_properties(torch.cuda.current_device()).total_memory
  weights = 2 * (sum(cfg.params_per_layer(i) for i in range(layers)) + 2 * cfg.vocab_size * cfg.hidden_size)
  per_tok = KVCache.bytes_per_page(cfg, layers) / 64
  pool_tokens = max(0.0, (total - weights - (4 << 30)) * 0.85) / per_tok
  return int(min(512 * world, max(64, pool_tokens // avg_ctx)))


def _serve_worker(rank: int, world: int, port: int, a: dict) -> None:
  import asyncio
  os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                    MASTER_PORT=str(port))
  from ..inference.shard import Shard
  from ..inference.tokenizers import _resolve_tokenizer
  from ..models import registry
  from ..models.config import load_config, preset
  from ..models.weights import load_hf_weights
  from ..runtime.runner import ShardRunner
  from ..train.ring_train import _model_dir
  from .comm import P2PTransport, init_distributed

  rank, world, dev = init_distributed()
  ctl = control_group() if world > 1 else None
  model = a["model"]
  mdir = _model_dir(model)
  cfg = load_config(mdir) if mdir is not None else preset(model)
  if not a.get("max_batch"):
    a = dict(a, max_batch=default_max_batch(cfg, world))

  def make_runner(r, w, group):
    shard = ring_shards(model, cfg.num_layers, w, group)[r]
    weights = (load_hf_weights(mdir, cfg, shard, dev)
               if mdir is not None and any(mdir.glob("*.safetensors")) else None)
    runner = ShardRunner(cfg, shard, dev, weights=weights, max_batch=a["max_batch"], max_ctx=a["max_ctx"], seed=0)
    print(f"[ring {r}/{w}] {model} layers {shard.start_layer}-{shard.end_layer} on {dev}"
          + ("" if weights is not None else " (random-init weights: no local checkpoint)"), flush=True)
    return runner, min_pool_pages(runner, w, group)

  runner, pool = make_runner(rank, world, ctl)
  monitor = HealthMonitor(rank, world).start() if world > 1 and os.environ.get("XOT_RING_HEALTH", "1") == "1" else None
  srv = RingServer(runner, rank, world, P2PTransport(rank, world, monitor=monitor), ctl, eos_ids=cfg.eos_token_ids,
                   monitor=monitor, make_runner=make_runner, pool_pages=pool)
  if rank == 0:
    tok = _resolve_tokenizer(mdir if mdir is not None else (registry.get_repo(model, "ShardedInferenceEngine") or "byte"),
                             cfg.vocab_size)
    full = Shard(model, 0, cfg.num_layers - 1, cfg.num_layers)
    asyncio.run(_rank0_main(srv, full, tok, cfg, a))
  else:
    srv.serve_forever()
  if dist.is_initialized():
    dist.destroy_process_group()


async def _rank0_main(srv: RingServer, shard, tok, cfg, a: dict) -> None:
  import asyncio
  loop = asyncio.get_running_loop()
  node = RingNode(srv, shard, tok, cfg.eos_token_ids, a["default_temp"], a["max_generate_tokens"], loop=loop,
                  config=cfg)
  viz = None
  if a.get("tui"):  # the reference's topology TUI, showing the GPU ring: one peer per rank, its layers, xGMI links
    try:
      from ..viz.topology_viz import TopologyViz
      viz = TopologyViz(chatgpt_api_endpoints=[f"http://localhost:{a['api_port']}/v1/chat/completions"],
                        web_chat_urls=[f"http://localhost:{a['api_port']}"], num_layers=cfg.num_layers)
      viz.update_visualization(node.current_topology, node.partitions, node.id, num_layers=cfg.num_layers)
      node.on_token.register("update_topology_viz").on_next(
        lambda rid, toks, fin: viz.update_prompt_output(rid, tok.decode(toks)))
    except Exception:
      viz = None
  th = threading.Thread(target=srv.serve_forever, name="xot-ring-rounds", daemon=True)
  th.start()
  try:
    if a.get("prompt") is not None:  # `xot run <model> --gpus N`: one prompt, print the answer
      done = asyncio.Event()
      out: List[int] = []

      def on_tok(rid, toks, fin):
        out.extend(toks)
        if fin:
          done.set()

      node.on_token.register("run").on_next(on_tok)
      # the same chat-templated prompt as the single-process `xot run` (main.run_model_cli)
      templ = tok.apply_chat_template([{"role": "user", "content": a["prompt"]}], tokenize=False,
                                      add_generation_prompt=True)
      await node.process_prompt(shard, templ, request_id="run-0",
                                inference_state={"max_tokens": a["max_generate_tokens"]})
      await asyncio.wait_for(done.wait(), timeout=600)
      print(tok.decode([t for t in out if t not in set(cfg.eos_token_ids)]), flush=True)
      return
    from ..api.chatgpt_api import ChatGPTAPI
    api = ChatGPTAPI(node, "ShardedInferenceEngine", response_timeout=a["response_timeout"],
                     default_model=a["model"], system_prompt=a.get("system_prompt"),
                     on_chat_completion_request=(lambda rid, req, prompt: viz.update_prompt(rid, prompt)) if viz else None)
    await api.run(port=a["api_port"])
    print(f"[ring 0] ChatGPT API on :{a['api_port']} (RCCL ring of {srv.world})", flush=True)
    if a.get("chat_tui"):
      from types import SimpleNamespace
      from ..viz.chat_tui import run_chat_tui
      await run_chat_tui(SimpleNamespace(default_model=a["model"], model_name=a["model"],
                                         chatgpt_api_response_timeout=a["response_timeout"]), api, node)
      return
    stop = asyncio.Event()  # SIGTERM / SIGINT: close the API, then stop the ring in order (exit code 0)
    import signal
    for sig in (signal.SIGINT, signal.SIGTERM):
      try:
        loop.add_signal_handler(sig, stop.set)
      except (NotImplementedError, RuntimeError):  # pragma: no cover
        pass
    await stop.wait()
    print("[ring 0] exit signal: shutting down", flush=True)
    await api.stop()
  finally:
    srv.stop()
    await asyncio.get_running_loop().run_in_executor(None, th.join, 60)


def serve_ring(args) -> int:
  """`xot [run] <model> --gpus N`: one process per GPU, continuous-batching ring over RCCL."""
  import torch.multiprocessing as mp
  from ..train.ring_train import _free_port
  n = args.gpus or max(1, torch.cuda.device_count())
  model = getattr(args, "model_name", None) or getattr(args, "run_model", None) or args.default_model
  a = {"model": model, "max_batch": int(os.environ.get("XOT_MAX_BATCH", 0)),  # 0: sized from HBM per rank
       "max_ctx": int(os.environ.get("XOT_MAX_CTX", 8192 if torch.cuda.is_available() else 2048)),
       "default_temp": args.default_temp, "max_generate_tokens": args.max_generate_tokens,
       "api_port": args.chatgpt_api_port, "response_timeout": args.chatgpt_api_response_timeout,
       "system_prompt": getattr(args, "system_prompt", None),
       "tui": not getattr(args, "disable_tui", True) and not getattr(args, "chat_tui", False) and sys.stdout.isatty(),
       "chat_tui": bool(getattr(args, "chat_tui", False)),
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

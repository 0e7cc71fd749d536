"""A local RCCL GPU ring as ONE peer of a discovered cluster (`xot --gpus N --federate`).

The reference's node always joins the discovered ring: discovery finds the peers, the partitioning strategy gives
each a layer range by memory, and activations hop peer to peer over gRPC (xotorch/main.py:143-173,
xotorch/orchestration/node.py:462-511 and 533-566); every peer also takes part in `xot train` through SendExample
(node.py:299-345, networking/grpc/grpc_server.py:94-114).  `xot --gpus N` alone serves the whole model on the box's
own RCCL ring (parallel/ring_serve.py), which no other host can join.  With --federate, rank 0 runs the ordinary
Node (gRPC server, UDP / manual discovery, ChatGPT API) whose capabilities are the sum of the box's GPUs, so the
partitioner hands the box a range sized for all of them; its engine is `RingFederatedEngine`, which splits whatever
range the cluster assigns over the local ranks and runs every step -- inference, training, evaluation, checkpoint
save / load -- through them, returning exactly what one engine holding the range would.

Control plane: rank 0 broadcasts a fixed int64 [op, payload bytes] header on the gloo control group, then the
payload as raw UTF-8 JSON (request ids, sub-ranges, prefix-cache operations); nothing is pickled.
Data plane: every hop is a fixed int64[8] word (ok, dtype, ndim, shape, numel) followed by the tensor's bytes on
that directed edge's own communicator (comm.P2PTransport: RCCL over xGMI on the box, gloo on CPU hosts).  A rank
whose step fails sends an error word with the message instead, every later rank passes it on, and rank 0 raises
it to the Node -- nobody waits forever on a dead step.

Serving is batched and pipelined: rank 0 cuts the steps queued on it into one batch, runs its sub-range (one
batched forward of its engine), broadcasts the batch header and hands the rows to rank 1, then goes on with the
next batch while the later ranks work on this one (at most `world` batches in flight); results come back from the
last rank in batch order on their own thread.  The prefix-cache operations of rank 0's first-layer cache (or the
ones arriving from the upstream peer) travel in the header, so every rank's KV pages follow the same forks.

Training / evaluation / checkpoints run exclusively (after the in-flight batches drain): forward rank to rank,
targets (or the downstream peer's gradient) from rank 0 to the last rank, loss back to rank 0, input gradients back
down the ring, then one AdamW step on every rank clipped by the norm over the whole box (the same numbers as one
engine holding the box's range).  Checkpoints are written per sub-range under the cluster's file naming, so they
form one partition that any other split can load (train/checkpoint.py).
"""
from __future__ import annotations

import asyncio
import functools
import json
import os
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path
from typing import List, Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist

from ..inference.inference_engine import InferenceEngine
from ..inference.shard import Shard
from .comm import P2PTransport

OP_STOP, OP_INFER, OP_FINISH, OP_TRAIN, OP_FWD, OP_SAVE, OP_LOAD = range(7)
_DTYPES = [torch.float32, torch.bfloat16, torch.int64, torch.int32, torch.float16, torch.uint8, torch.float64]


class FederationError(RuntimeError):
  """A step failed on a rank of the local ring (the message names the rank and the error)."""


def split_shard(shard: Shard, world: int) -> List[Shard]:
  """The layer range of `shard` in `world` contiguous, near-equal sub-ranges (at most one per layer)."""
  n = shard.end_layer - shard.start_layer + 1
  parts = min(world, n)
  out, start = [], shard.start_layer
  for r in range(parts):
    k = n // parts + (1 if r < n % parts else 0)
    out.append(Shard(shard.model_id, start, start + k - 1, shard.n_layers))
    start += k
  return out


def federation_edges(world: int) -> list:
  """Directed edges the local ring uses, each its own communicator: r -> r+1 (activations), r+1 -> r (input
  gradients), r -> 0 (results, losses) and 0 -> r (targets / the downstream gradient for the last sub-range)."""
  edges = []
  for e in [e for r in range(world - 1) for e in ((r, r + 1), (r + 1, r))] + \
           [e for r in range(1, world) for e in ((r, 0), (0, r))]:
    if e not in edges:
      edges.append(e)
  return edges


class Wire:
  """Headers on the control group, tensors with their fixed-size meta word on the edge communicators."""

  def __init__(self, rank: int, world: int, groups: dict, device: torch.device):
    self.rank, self.world = rank, world
    self.ctl = groups["ctl"]
    self.dev = device
    self.t = P2PTransport(rank, world, edges=federation_edges(world))
    self.on = device if (device.type == "cuda" and not self.t._staged) else torch.device("cpu")

  # ---------------------------------------------------------------- control
  def header(self, op: int, payload: Optional[dict] = None) -> None:
    raw = json.dumps(payload or {}, separators=(",", ":")).encode()
    dist.broadcast(torch.tensor([op, len(raw)], dtype=torch.int64), 0, group=self.ctl)
    dist.broadcast(torch.frombuffer(bytearray(raw), dtype=torch.uint8), 0, group=self.ctl)

  def get_header(self) -> Tuple[int, dict]:
    h = torch.empty(2, dtype=torch.int64)
    dist.broadcast(h, 0, group=self.ctl)
    raw = torch.empty(int(h[1]), dtype=torch.uint8)
    dist.broadcast(raw, 0, group=self.ctl)
    return int(h[0]), json.loads(raw.numpy().tobytes())

  def allreduce(self, t: torch.Tensor) -> torch.Tensor:
    """Sum over every rank (host tensors on the control group); returns it on t's device."""
    h = t.detach().to("cpu", copy=True)
    dist.all_reduce(h, group=self.ctl)
    return h.to(t.device)

  # ---------------------------------------------------------------- data
  def put(self, t: Optional[torch.Tensor], dst: int, err: Optional[str] = None) -> None:
    """Send t to dst, or (err given / no tensor) an error word carrying the message."""
    if err is not None or t is None:
      raw = (err or "no tensor").encode()[:4000]
      self.t.isend(torch.tensor([0, 0, 0, 0, 0, 0, 0, len(raw)], dtype=torch.int64, device=self.on), dst)
      self.t.isend(torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(self.on), dst)
      return
    t = t.detach().contiguous()
    if t.dim() > 4:
      raise ValueError(f"hop tensors have at most 4 dims, got {tuple(t.shape)}")
    meta = [1, _DTYPES.index(t.dtype), t.dim()] + list(t.shape) + [0] * (4 - t.dim()) + [t.numel()]
    self.t.isend(torch.tensor(meta, dtype=torch.int64, device=self.on), dst)
    if t.device != self.on and not (t.is_cuda and self.t._staged):
      t = t.to(self.on)
    self.t.isend(t.view(torch.int16) if t.dtype == torch.bfloat16 else t, dst)

  def get(self, src: int) -> Tuple[Optional[torch.Tensor], Optional[str]]:
    """(tensor on this rank's device, None) or (None, the error message an upstream rank sent)."""
    meta = torch.empty(8, dtype=torch.int64, device=self.on)
    self.t.recv(meta, src)
    m = meta.tolist()
    if m[0] == 0:
      raw = torch.empty(m[7], dtype=torch.uint8, device=self.on)
      self.t.recv(raw, src)
      return None, raw.cpu().numpy().tobytes().decode(errors="replace")
    dt = _DTYPES[m[1]]
    buf = torch.empty(m[3:3 + m[2]], dtype=torch.int16 if dt == torch.bfloat16 else dt, device=self.dev)
    self.t.recv(buf, src)
    return (buf.view(torch.bfloat16) if dt == torch.bfloat16 else buf), None

  def recv(self, src: int) -> torch.Tensor:
    t, err = self.get(src)
    if err is not None:
      raise FederationError(err)
    return t

  def drain(self) -> None:
    self.t.drain()


def _err(rank: int, e: BaseException) -> str:
  return f"rank {rank}: {type(e).__name__}: {e}"


def _as_tensor(x) -> torch.Tensor:
  return x.detach() if isinstance(x, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(np.asarray(x)))


# ------------------------------------------------------------------ one rank's part of a training step
def _tied_shape(tr) -> Optional[list]:
  """[V, D] when the box holds both ends of a tied-embedding model (rank 0's embed, the last rank's head copy)."""
  return list(tr.params["embed"].shape) if (tr.c.tie_word_embeddings and "embed" in tr.params) else None


def stage_train(tr, w: Wire, r: int, n: int, mode: str, tied: Optional[list], x=None, target=None, length=None):
  """Rank r's share of one train ("ce": the box ends the model / "bg": the downstream peer's gradient) or evaluate
  ("eval") step over sub-ranges 0..n-1.  Every message slot of the protocol is always filled (data or an error
  word), and every rank joins the control-group reductions, so a failure anywhere ends the step everywhere.
  Returns (loss, grad wrt the box's input) on rank 0 (raises FederationError if any rank failed)."""
  err = None
  last = r == n - 1
  train = mode != "eval"
  tgt = lens = None
  if r > 0 and r < n:
    x, err = w.get(r - 1)
  if last and r < n:
    tgt, e = w.get(0)
    err = err or e
    if mode != "bg":
      lens, e = w.get(0)
      err = err or e
  leaf = out = None
  if r < n and err is None:
    try:
      if train:
        tr.zero_grad()
        leaf, out = tr.forward_train(x)
      else:
        with torch.no_grad():
          out = tr.forward(tr._to(x))
    except Exception as e:  # noqa: BLE001 - sent on, raised on rank 0
      err = _err(r, e)
  if r < n and not last:
    w.put(None if err else out.detach().to(torch.bfloat16), r + 1, err)
  if r == 0:  # the last sub-range's targets (or the downstream gradient), after the activation
    if mode == "bg":
      w.put(_as_tensor(target).to(torch.bfloat16), n - 1)
    else:
      w.put(_as_tensor(target).to(torch.int64), n - 1)
      w.put(_as_tensor(length).to(torch.int64).view(-1), n - 1)
  loss, gin = 0.0, None
  if last and r < n:
    if err is None:
      try:
        if mode == "bg":
          _, gin = tr.backward_accumulate(leaf, out, grad_out=tgt)
        else:
          L = tgt.shape[1]
          denom = float(max(int(lens.clamp(max=L).sum()), 1))
          if train:
            lt, gin = tr.backward_accumulate(leaf, out, target=tgt, length=lens, denom=denom)
            loss = float(lt)
          else:
            loss = float(tr.loss_of(out, tgt, lens)[0])
      except Exception as e:  # noqa: BLE001
        err = _err(r, e)
    w.put(None if err else torch.tensor([loss], dtype=torch.float64), 0, err)
  if r == 0:
    lt, e = w.get(n - 1)
    err = err or e
    loss = float(lt[0]) if lt is not None else 0.0
  if train and r < n and not last:
    g, e = w.get(r + 1)
    err = err or e
    if err is None:
      try:
        _, gin = tr.backward_accumulate(leaf, out, grad_out=g)
      except Exception as ex:  # noqa: BLE001
        err = _err(r, ex)
  if train and 0 < r < n:
    w.put(None if err else gin.to(torch.bfloat16), r - 1, err)
  # one verdict for the whole box: the step applies everywhere or nowhere
  bad = w.allreduce(torch.tensor([0.0 if err is None else 1.0], dtype=torch.float64))
  if train and float(bad[0]) == 0.0:
    exclude = ()
    if tied is not None:  # both ends of a tied embedding on this box: sum the two copies' gradients
      name = "embed" if r == 0 else ("lm_head" if last and r < n else None)
      g = tr.grads().get(name) if name else None
      g = torch.zeros(tied, dtype=torch.float32) if g is None else g.float()
      g = w.allreduce(g)
      if name is not None:
        acc = tr.acc.get(name)
        if acc is not None:
          acc.buf.copy_(g)
          acc.fresh = False
        else:
          tr.params[name].grad = g.to(tr.params[name].dtype)
      exclude = ("lm_head",) if last else ()
    if r < n:
      tr.apply(grad_norm_sq_reduce=w.allreduce, norm_exclude=exclude)
    else:  # idle rank: its share of the norm reduction
      w.allreduce(torch.zeros(1))
  if r == 0 and err is not None:
    raise FederationError(err)
  if r == 0 and float(bad[0]) != 0.0:
    raise FederationError("a rank of the local ring failed the step")
  return loss, (gin.detach().cpu() if gin is not None else None)


def stage_forward(tr, w: Wire, r: int, n: int, x=None):
  """train_forward / eval_forward over the local ring: the box's output activation, on rank 0."""
  err = None
  if r >= n:
    return None
  if r > 0:
    x, err = w.get(r - 1)
  out = None
  if err is None:
    try:
      with torch.no_grad():
        out = tr.forward(tr._to(x))
    except Exception as e:  # noqa: BLE001
      err = _err(r, e)
  w.put(None if err else out, r + 1 if r < n - 1 else 0, err)
  if r == 0:
    return w.recv(n - 1).cpu()
  return None


def _checkpoint_parts(path: str, subs: List[Shard]) -> List[str]:
  """The per-sub-range file names of a checkpoint the Node asked for under `path` (train/checkpoint.py names)."""
  from ..train.checkpoint import _NAME, checkpoint_path
  p = Path(path)
  m = _NAME.match(p.name)
  if m is None:
    raise ValueError(f"{path}: not a checkpoint file name (<dir>/<model>/SSS-EEE-of-NNN-IIIIII.safetensors)")
  return [str(checkpoint_path(p.parent.parent, s, int(m.group(4)))) for s in subs]


# ------------------------------------------------------------------ rank 0
class RingFederatedEngine(InferenceEngine):
  """Rank 0's engine: the Node's shard split over the local ring (module docstring)."""

  def __init__(self, local, rank: int, world: int, groups: dict, device: torch.device):
    self.local = local  # ShardedInferenceEngine of rank 0's sub-range
    self.rank, self.world = rank, world
    self.device = device
    self.wire = Wire(rank, world, groups, device) if world > 1 else None
    self.shard: Optional[Shard] = None
    self._queue: list = []  # (rid, shard, input, state, future) waiting for the next batch
    self._draining = False
    self._inflight = 0
    self._idle: Optional[asyncio.Event] = None
    self._gate: Optional[asyncio.Lock] = None  # batch launches vs. exclusive operations
    self._slots: Optional[asyncio.Semaphore] = None
    # one thread sends (headers, hops, exclusive operations), one receives batch results: each edge then
    # carries one ordered stream, and a result wait never holds up the next batch's hand-off
    self._tx = ThreadPoolExecutor(max_workers=1, thread_name_prefix="xot-fed-tx")
    self._rx = ThreadPoolExecutor(max_workers=1, thread_name_prefix="xot-fed-rx")
    self.stats = {"batches": 0, "requests": 0}

  def _sync_objs(self):
    if self._gate is None:
      self._gate, self._idle, self._slots = asyncio.Lock(), asyncio.Event(), asyncio.Semaphore(max(1, self.world))
      self._idle.set()

  # the Node reads these off its engine (EOS handling, token text for the TUI)
  @property
  def tokenizer(self):
    return getattr(self.local, "tokenizer", None)

  @property
  def eos_token_ids(self):
    return getattr(self.local, "eos_token_ids", ())

  async def _on(self, pool, fn, *args, **kw):
    return await asyncio.get_running_loop().run_in_executor(pool, functools.partial(fn, *args, **kw))

  async def encode(self, shard: Shard, prompt: str) -> np.ndarray:
    return await self.local.encode(split_shard(shard, self.world)[0], prompt)

  async def decode(self, shard: Shard, tokens: np.ndarray) -> str:
    return await self.local.decode(split_shard(shard, self.world)[0], tokens)

  async def sample(self, x, temp: float = 0.0, top_k: int = 35) -> np.ndarray:
    return await self.local.sample(x, temp=temp, top_k=top_k)

  async def infer_prompt(self, request_id: str, shard: Shard, prompt: str,
                         inference_state: Optional[dict] = None) -> Tuple[object, Optional[dict]]:
    ids = await self.encode(shard, prompt)
    return await self.infer_tensor(request_id, shard, np.asarray(ids).reshape(1, -1), inference_state)

  # ---------------------------------------------------------------- batched, pipelined inference
  async def infer_tensor(self, request_id: str, shard: Shard, input_data,
                         inference_state: Optional[dict] = None) -> Tuple[object, Optional[dict]]:
    subs = split_shard(shard, self.world)
    self.shard = shard
    if len(subs) == 1:
      return await self.local.infer_tensor(request_id, subs[0], input_data, inference_state)
    self._sync_objs()
    fut = asyncio.get_running_loop().create_future()
    self._queue.append((request_id, shard, input_data, inference_state or {}, fut))
    if not self._draining:
      self._draining = True
      asyncio.create_task(self._drain())
    return await fut

  def _cut(self) -> list:
    """The next batch: queued steps of the first one's shard, one per request."""
    if not self._queue:
      return []
    shard = self._queue[0][1]
    batch, rest, seen = [], [], set()
    for it in self._queue:
      if it[1] == shard and it[0] not in seen:
        batch.append(it)
        seen.add(it[0])
      else:
        rest.append(it)
    self._queue = rest
    return batch

  async def _drain(self):
    try:
      while self._queue:
        for _ in range(4):  # the follow-up steps of one Node round arrive through a few tasks: let them queue
          await asyncio.sleep(0)
        await self._slots.acquire()
        async with self._gate:
          batch = self._cut()
          if not batch:
            self._slots.release()
            continue
          self._inflight += 1
          self._idle.clear()
          try:
            await self._launch(batch)
          except BaseException as e:  # noqa: BLE001 - delivered to the batch's waiters
            for it in batch:
              if not it[4].done():
                it[4].set_exception(e)
            self._retire()
    finally:
      self._draining = False

  def _retire(self) -> None:
    self._inflight -= 1
    if self._inflight == 0:
      self._idle.set()
    self._slots.release()

  async def _launch(self, batch: list) -> None:
    subs = split_shard(batch[0][1], self.world)
    outs = await asyncio.gather(*(self.local.infer_tensor(rid, subs[0], x, st) for rid, _, x, st, _ in batch),
                                return_exceptions=True)
    good = []
    for it, o in zip(batch, outs):
      if isinstance(o, BaseException):
        it[4].set_exception(o)
      else:
        good.append((it, o))
    if not good:
      self._retire()
      return
    rows, qlens, ops = [], [], []
    for (rid, _, x, st_in, _), (y, st) in good:
      y = _as_tensor(y)
      L = y.shape[1]
      rows.append(y.reshape(L, -1))
      qlens.append(L)
      # KV page operations every rank must mirror: those of rank 0's own first-layer cache, or the upstream's
      ops.append((st or {}).get("pc") if subs[0].is_first_layer() else st_in.get("pc"))
    payload = {"rids": [it[0] for it, _ in good], "qlens": qlens, "subs": [s.to_dict() for s in subs], "pc": ops}
    x = torch.cat(rows).to(self.device, torch.bfloat16)
    self.stats["batches"] += 1
    self.stats["requests"] += len(good)
    loop = asyncio.get_running_loop()
    # submitted now, in batch order (a coroutine wrapper would submit only when its task first runs)
    tx = loop.run_in_executor(self._tx, self._send_batch, payload, x)
    rx = loop.run_in_executor(self._rx, self.wire.recv, len(subs) - 1)
    asyncio.create_task(self._collect(tx, rx, good, qlens, subs[-1].is_last_layer()))

  def _send_batch(self, payload: dict, x: torch.Tensor) -> None:
    self.wire.header(OP_INFER, payload)
    self.wire.put(x, 1)

  async def _collect(self, tx, rx, good, qlens, logits: bool) -> None:
    try:
      await tx
      out = await rx
      off = 0
      for i, ((_, _, _, _, fut), (_, st)) in enumerate(good):
        if logits:  # [n, V] fp32 on this device: each request's last-token row, ready for the sampler
          r = out[i:i + 1]
        else:
          r = out[off:off + qlens[i]].reshape(1, qlens[i], -1).cpu()
          off += qlens[i]
        if not fut.done():
          fut.set_result((r, st))
    except BaseException as e:  # noqa: BLE001
      for (_, _, _, _, fut), _ in good:
        if not fut.done():
          fut.set_exception(e)
    finally:
      self._retire()

  async def finish_request(self, request_id: str, ok: bool = True) -> None:
    if self.world > 1:  # after every batch already handed on (the send thread's order)
      await self._on(self._tx, self.wire.header, OP_FINISH, {"rid": request_id, "ok": ok})
    await self.local.finish_request(request_id, ok=ok)

  async def ensure_shard(self, shard: Shard):
    await self.local.ensure_shard(split_shard(shard, self.world)[0])

  # ---------------------------------------------------------------- exclusive operations
  async def _exclusive(self, fn, *args):
    self._sync_objs()
    async with self._gate:
      await self._idle.wait()
      return await self._on(self._tx, fn, *args)

  async def train(self, request_id: str, shard: Shard, example, target, length, train: bool = True,
                  loss: str = "length_masked_ce"):
    subs = split_shard(shard, self.world)
    self.shard = shard
    if len(subs) == 1:
      return await self.local.train(request_id, subs[0], example, target, length, train=train, loss=loss)
    await self.local.ensure_shard(subs[0])
    mode = "eval" if not train else ("bg" if loss == "back_gradient" else "ce")
    res = await self._exclusive(self._root_train, request_id, subs, example, target, length, mode)
    return res[0] if mode == "eval" else res

  async def evaluate(self, request_id: str, shard: Shard, example, target, length, loss: str = "length_masked_ce"):
    return await self.train(request_id, shard, example, target, length, train=False, loss=loss)

  def _root_train(self, rid, subs, example, target, length, mode):
    tr = self.local._get_trainer()
    x = _as_tensor(example)
    tied = _tied_shape(tr) if subs[-1].is_last_layer() and subs[0].is_first_layer() else None
    self.wire.header(OP_TRAIN, {"rid": rid, "subs": [s.to_dict() for s in subs], "mode": mode, "tied": tied})
    return stage_train(tr, self.wire, 0, len(subs), mode, tied, x=x, target=target, length=length)

  async def train_forward(self, request_id: str, shard: Shard, example):
    subs = split_shard(shard, self.world)
    if len(subs) == 1:
      return await self.local.train_forward(request_id, subs[0], example)
    await self.local.ensure_shard(subs[0])
    return await self._exclusive(self._root_forward, subs, example)

  async def eval_forward(self, request_id: str, shard: Shard, example):
    return await self.train_forward(request_id, shard, example)

  def _root_forward(self, subs, example):
    self.wire.header(OP_FWD, {"subs": [s.to_dict() for s in subs]})
    return stage_forward(self.local._get_trainer(), self.wire, 0, len(subs), x=_as_tensor(example))

  async def save_checkpoint(self, shard: Shard, path: str):
    subs = split_shard(shard, self.world)
    if len(subs) == 1:
      return await self.local.save_checkpoint(subs[0], path)
    from ..train.checkpoint import save_shard_checkpoint
    parts = _checkpoint_parts(path, subs)
    await self.local.ensure_shard(subs[0])
    await self._exclusive(self._root_checkpoint, OP_SAVE, {"subs": [s.to_dict() for s in subs], "paths": parts},
                          functools.partial(save_shard_checkpoint, self.local, subs[0], parts[0]))

  async def load_checkpoint(self, shard: Shard, path: str):
    subs = split_shard(shard, self.world)
    if len(subs) == 1:
      return await self.local.load_checkpoint(subs[0], path)
    from ..train.checkpoint import load_shard_checkpoint
    await self.local.ensure_shard(subs[0])
    await self._exclusive(self._root_checkpoint, OP_LOAD, {"subs": [s.to_dict() for s in subs], "path": str(path)},
                          functools.partial(load_shard_checkpoint, self.local, subs[0], path))

  def _root_checkpoint(self, op: int, payload: dict, fn) -> None:
    """Header, rank 0's own part, then one verdict over every rank -- a single job on the send thread, so no
    other header can come between them."""
    self.wire.header(op, payload)
    err = None
    try:
      fn()
    except Exception as e:  # noqa: BLE001
      err = e
    bad = self.wire.allreduce(torch.tensor([0.0 if err is None else 1.0]))
    if err is not None:
      raise err
    if float(bad[0]):
      raise FederationError(f"{int(bad[0])} rank(s) of the local ring failed the checkpoint operation")

  def stop(self) -> None:
    if self.world > 1:
      self._tx.submit(self.wire.header, OP_STOP).result()
      self.wire.drain()


# ------------------------------------------------------------------ ranks 1..N-1
async def follower_loop(local, rank: int, world: int, groups: dict, device: torch.device) -> None:
  """Ranks 1..N-1: act on rank 0's headers until "stop"."""
  wire = Wire(rank, world, groups, device)
  loop = asyncio.get_running_loop()
  io = ThreadPoolExecutor(max_workers=1, thread_name_prefix="xot-fed-io")

  async def on_io(fn, *a):
    return await loop.run_in_executor(io, functools.partial(fn, *a))

  while True:
    op, p = await on_io(wire.get_header)
    if op == OP_STOP:
      wire.drain()
      return
    if op == OP_FINISH:
      await local.finish_request(p["rid"], ok=p.get("ok", True))
      continue
    subs = [Shard.from_dict(s) for s in p["subs"]]
    n = len(subs)
    if op == OP_INFER:
      if rank < n:
        await _follow_infer(local, wire, rank, subs, p, on_io, device)
    elif op in (OP_TRAIN, OP_FWD):
      tr, err = None, None
      if rank < n:
        try:
          await local.ensure_shard(subs[rank])
          tr = await local._run(local._get_trainer)
        except Exception as e:  # noqa: BLE001 - the stage then reports it through the protocol
          err = e
      if op == OP_FWD:
        await on_io(stage_forward, _Broken(err) if err else tr, wire, rank, n)
      else:
        await on_io(stage_train, _Broken(err) if err else tr, wire, rank, n, p["mode"], p.get("tied"))
    elif op in (OP_SAVE, OP_LOAD):
      err = None
      if rank < n:
        try:
          if op == OP_SAVE:
            await local.save_checkpoint(subs[rank], p["paths"][rank])
          else:
            await local.load_checkpoint(subs[rank], p["path"])
        except Exception as e:  # noqa: BLE001
          err = e
          print(f"[federate rank {rank}] checkpoint operation failed: {e}")
      await on_io(wire.allreduce, torch.tensor([0.0 if err is None else 1.0]))


class _Broken:
  """A trainer that could not be built: every use raises the original error (reported through the protocol)."""

  def __init__(self, err: BaseException):
    self.err = err

  def __getattr__(self, name):
    raise self.err


async def _follow_infer(local, wire: Wire, rank: int, subs: List[Shard], p: dict, on_io, device) -> None:
  n = len(subs)
  nxt = rank + 1 if rank + 1 < n else 0
  x, err = await on_io(wire.get, rank - 1)
  if err is None:
    try:
      sub = subs[rank]
      steps, off = [], 0
      for rid, L, ops in zip(p["rids"], p["qlens"], p["pc"]):
        steps.append(local.infer_tensor(rid, sub, x[off:off + L].reshape(1, L, -1), {"pc": ops} if ops else {}))
        off += L
      outs = await asyncio.gather(*steps)
      if sub.is_last_layer():
        y = torch.cat([_as_tensor(o[0]).reshape(1, -1).to(device, torch.float32) for o in outs])
      else:
        y = torch.cat([_as_tensor(o[0]).reshape(-1, x.shape[-1]) for o in outs]).to(device, torch.bfloat16)
    except Exception as e:  # noqa: BLE001 - the error word travels on to rank 0
      err = _err(rank, e)
  await on_io(wire.put, None if err else y, nxt, err)


def ring_capabilities(world: int):
  """The box as one peer: every local GPU's memory and FLOPS summed (so the cluster partitioner sizes its
  layer range for the whole ring)."""
  from ..topology.device_capabilities import DeviceCapabilities, DeviceFlops, device_capabilities
  one = device_capabilities()
  f = one.flops
  return DeviceCapabilities(model=f"{one.model} x{world} (RCCL ring)", chip=one.chip, memory=one.memory * world,
                            flops=DeviceFlops(fp32=f.fp32 * world, fp16=f.fp16 * world, int8=f.int8 * world))


def _federate_worker(rank: int, world: int, port: int, argv: List[str]) -> None:
  os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                    MASTER_PORT=str(port), XOT_PEER_RANK=str(rank))
  from ..download.new_shard_download import new_shard_downloader
  from ..inference.sharded_engine import ShardedInferenceEngine
  from .comm import init_distributed
  from .ring_serve import control_group
  from .. import main as xot_main

  rank, world, dev = init_distributed()
  groups = {"ctl": control_group(), "data": dist.group.WORLD}
  args = xot_main.build_parser().parse_args(argv)
  local = ShardedInferenceEngine(new_shard_downloader(args.max_parallel_downloads), device=dev)
  try:
    if rank == 0:
      engine = RingFederatedEngine(local, rank, world, groups, dev)
      rc = asyncio.run(xot_main.async_main(args, engine=engine, device_caps=ring_capabilities(world)))
      engine.stop()
    else:
      asyncio.run(follower_loop(local, rank, world, groups, dev))
      rc = 0
  finally:
    if dist.is_initialized():
      dist.destroy_process_group()
  raise SystemExit(rc or 0)


def worker_argv(argv: List[str]) -> List[str]:
  """The command line of a rank: the user's, without --gpus N / --federate (each rank is one process)."""
  rest, skip = [], False
  for a in argv:
    if skip:
      skip = False
      continue
    if a in ("--gpus", "--federate") or a.startswith("--gpus="):
      skip = a == "--gpus"
      continue
    rest.append(a)
  return rest


def federate_ring(args, argv: List[str]) -> int:
  """`xot --gpus N --federate`: one process per local GPU; rank 0 is the cluster peer (module docstring)."""
  import torch.multiprocessing as mp
  from ..train.ring_train import _free_port
  n = args.gpus
  port = _free_port()
  rest = worker_argv(argv)
  ctx = mp.get_context("spawn")
  procs = [ctx.Process(target=_federate_worker, args=(r, n, port, rest)) for r in range(n)]
  for p in procs:
    p.start()
  rc = 0
  for p in procs:
    p.join()
    rc = rc or (p.exitcode or 0)
  return rc

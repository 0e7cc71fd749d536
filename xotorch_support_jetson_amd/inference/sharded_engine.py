"""ShardedInferenceEngine: the MI355X engine behind the Node (reference: TorchDynamicShardInferenceEngine,
xotorch/inference/torch/sharded_inference_engine.py:37-424).

Differences by design:
  * one ShardRunner per shard: HIP kernels, paged per-request KV (concurrent requests do not clobber
    each other as they do in the reference's single global cache), HIP-graph decode;
  * the inference state shipped between peers is {"n_past": int} — positions and masks are derived
    on the device (the reference JSON-ships tokens, positions and a [1,T,T] mask on every hop);
  * hidden states travel as bf16 tensors; the last shard returns fp32 logits of the last token only;
  * per-request temperature reaches the sampler (the reference drops the API temperature).
Weights come from a local HF snapshot of the shard when present (safetensors, this shard's tensors
only) and otherwise from the deterministic random init of the exact architecture (offline boxes).
"""
from __future__ import annotations

import asyncio
import os
import time
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path
from typing import Optional, Tuple

import numpy as np
import torch

from ..helpers import DEBUG
from ..models import registry
from ..models.config import ModelConfig, load_config, preset
from .inference_engine import InferenceEngine
from .shard import Shard
from .tokenizers import _resolve_tokenizer

TEMPERATURE = 0.6
TOP_K = 35


def _temp_of(state: dict) -> float:
  """A request's sampling temperature; a key present as None (the API's "not given") means the default."""
  t = state.get("temperature")
  return TEMPERATURE if t is None else float(t)


def default_device() -> torch.device:
  env = os.environ.get("TORCH_DEVICE") or os.environ.get("XOT_DEVICE")
  if env:
    return torch.device(env)
  if torch.cuda.is_available():
    return torch.device("cuda", int(os.environ.get("LOCAL_RANK", 0)) % max(1, torch.cuda.device_count()))
  return torch.device("cpu")


# new tokens per batched forward (prefill chunks + decode tokens): bounds the step's activations and keeps a
# burst of long prompts from stalling every decoding request for one huge step (vLLM's max_num_batched_tokens)
MAX_STEP_TOKENS = int(os.environ.get("XOT_MAX_STEP_TOKENS", "8192"))
PRESAMPLE = os.environ.get("XOT_PRESAMPLE", "1") == "1"
# prompt-prefix KV reuse (inference/prefix_cache.py): on by default, at most this fraction of the KV pool
PREFIX_CACHE = os.environ.get("XOT_PREFIX_CACHE", "1") == "1"
PREFIX_CACHE_FRAC = float(os.environ.get("XOT_PREFIX_CACHE_FRAC", "0.25"))
# single-peer requests decode in the engine's own loop (continue_locally); 0 = one Node round trip per token
ENGINE_LOOP = os.environ.get("XOT_ENGINE_LOOP", "1") == "1"
# engine-loop decode steps chained on the device: step N+1 takes step N's sampled ids straight from device
# memory and is queued before step N's tokens reach the host (no GPU idle gap between decode steps)
CHAIN = os.environ.get("XOT_CHAIN", "1") == "1"
# diagnostics: time chained steps on the GPU with events (stats gpu_step_s / gpu_gap_s)
STEP_EVENTS = os.environ.get("XOT_STEP_EVENTS", "0") == "1"


class ShardedInferenceEngine(InferenceEngine):
  def __init__(self, shard_downloader=None, device: Optional[torch.device] = None, seed: int = 1234):
    self.shard: Optional[Shard] = None
    self.shard_downloader = shard_downloader
    self.device = device or default_device()
    self.executor = ThreadPoolExecutor(max_workers=1, thread_name_prefix="xot-engine")
    self.runner = None
    self.config: Optional[ModelConfig] = None
    self.tokenizer = None
    self.model_path: Optional[Path] = None
    self.seed = seed
    self.seed_off = torch.tensor([seed, 0], dtype=torch.int64)
    self._lock = asyncio.Lock()
    self.trainer = None
    self.lr = float(os.environ.get("XOT_LR", "1e-5"))  # `xot train --lr` sets this
    self._queue: list = []  # (request id, shard, input, future) waiting for the next batched step
    self._draining = False
    self._images: dict = {}  # request id -> [N, 3, S, S] pixels awaiting that request's prefill (LLaVA)
    self._sample_q: list = []  # (logits, temperature, top_k, future) drawn together by _drain_samples
    self._sampling = False
    self.stats = {"steps": 0, "requests": 0, "tokens": 0}  # batched forward steps (serving diagnostics)
    self._presampled: dict = {}  # (logits ptr, row) -> (temperature, top_k, token) drawn with the forward
    self._presampled_prev: dict = {}  # the step before's (the next step may start before its readers sample)
    self.prefix_cache = None  # first shard's PrefixCache (built with the runner)
    self._loops: dict = {}  # request id -> (emit, fail, stop) of requests decoding in the engine loop

  # ------------------------------------------------------------------ helpers
  async def _run(self, fn, *args):
    return await asyncio.get_running_loop().run_in_executor(self.executor, fn, *args)

  async def encode(self, shard: Shard, prompt: str) -> np.ndarray:
    await self.ensure_shard(shard)
    ids = self.tokenizer.encode(prompt)
    return np.asarray(ids, dtype=np.int64)

  async def decode(self, shard: Shard, tokens: np.ndarray) -> str:
    await self.ensure_shard(shard)
    return self.tokenizer.decode(np.asarray(tokens).reshape(-1).tolist())

  def _seed(self, dev: torch.device) -> torch.Tensor:
    """[seed, offset] for the sampler on `dev`, advanced after each use by _advance_seed.  On a GPU it lives
    on the device (advanced by a tiny kernel), so a sampler launch never waits on a host-to-device copy."""
    if dev.type != "cuda":
      return self.seed_off
    t = getattr(self, "_seed_dev", None)
    if t is None or t.device != dev:
      t = self._seed_dev = self.seed_off.to(dev)
    return t

  def _advance_seed(self, dev: torch.device) -> None:
    self.seed_off[1] += 1
    if dev.type == "cuda":
      self._seed(dev)[1:].add_(1)

  @staticmethod
  def _temps(values: list, dev: torch.device) -> torch.Tensor:
    """Per-row temperatures on `dev` without a blocking copy (one fill kernel when they are all equal)."""
    if dev.type != "cuda":
      return torch.tensor(values, dtype=torch.float32)
    if all(v == values[0] for v in values):
      return torch.full((len(values),), values[0], dtype=torch.float32, device=dev)
    return torch.tensor(values, dtype=torch.float32).pin_memory().to(dev, non_blocking=True)

  def _presample(self, logits: torch.Tensor, states: list) -> None:
    """Last shard: draw the step's tokens right after its forward, in the same executor call (one
    sampler launch, one device-to-host copy), for requests whose state carries their sampling
    parameters (the Node forwards temperature / top_k with every step).  sample() then returns the
    stored token without another trip through the executor."""
    # tokens of the step before last nobody asked for (finished requests) go; the last step's stay one more
    # step, since with the pipelined engine loop this step may have started before that step's Node-path
    # readers sampled.  A lagging request still holds its logits view, so no new tensor can reuse that base
    # address and collide with a fresh key
    self._presampled_prev, self._presampled = self._presampled, {}
    if not PRESAMPLE or not states or any(st.get("temperature") is None for st in states):
      return
    from ..ops import kernels as K
    groups = {}
    for i, st in enumerate(states):
      groups.setdefault(int(st.get("top_k") or TOP_K), []).append(i)
    for k, idx in groups.items():
      dev = logits.device
      sel = logits if len(idx) == logits.shape[0] else logits[torch.tensor(idx).to(dev, non_blocking=True)]
      temps = self._temps([_temp_of(states[i]) for i in idx], dev)
      tok = K.sample(sel.contiguous(), temps, k, self._seed(dev))
      self._advance_seed(dev)
      tok = tok.cpu().numpy().astype(np.int64)  # the step's one blocking point
      for j, i in enumerate(idx):
        self._presampled[(logits.data_ptr(), i)] = (_temp_of(states[i]), k, tok[j:j + 1])

  async def sample(self, x, temp: float = TEMPERATURE, top_k: int = TOP_K) -> np.ndarray:
    """Sample one request's next token.  A token drawn with the forward (_presample, same parameters)
    is returned at once; otherwise concurrent calls (the requests of one batched step) are drawn
    together: one sampler launch over their stacked logits and one device-to-host copy, instead of a
    launch + synchronisation per request."""
    if isinstance(x, torch.Tensor) and x.dim() == 2 and x.shape[0] == 1 and (self._presampled or self._presampled_prev):
      key = self._presample_key(x)
      hit = None
      if key is not None:
        hit = self._presampled.pop(key, None)
        if hit is None:
          hit = self._presampled_prev.pop(key, None)
      if hit is not None and hit[0] == float(temp) and hit[1] == int(top_k):
        self.stats["presampled"] = self.stats.get("presampled", 0) + 1
        return hit[2]
    fut = asyncio.get_running_loop().create_future()
    self._sample_q.append((x, float(temp), int(top_k), fut))
    if not self._sampling:
      self._sampling = True
      asyncio.create_task(self._drain_samples())
    return await fut

  @staticmethod
  def _presample_key(x: torch.Tensor):
    """(data pointer of the step's logits tensor, row) of a [1, V] row view of it."""
    if x._base is None or x._base.dim() != 2:
      return None
    row = (x.data_ptr() - x._base.data_ptr()) // (x.element_size() * x._base.stride(0))
    return (x._base.data_ptr(), int(row))

  async def _drain_samples(self):
    try:
      while self._sample_q:
        batch, self._sample_q = self._sample_q, []
        try:
          res = await self._run(self._sample_batch, [(x, t, k) for x, t, k, _ in batch])
          for (_, _, _, fut), r in zip(batch, res):
            if not fut.done():
              fut.set_result(r)
        except Exception as e:  # noqa: BLE001 - delivered to every waiter
          for *_, fut in batch:
            if not fut.done():
              fut.set_exception(e)
    finally:
      self._sampling = False

  def _sample_batch(self, items):
    from ..ops import kernels as K
    rows, out = [], [None] * len(items)
    for x, _, _ in items:
      t = torch.as_tensor(x) if not isinstance(x, torch.Tensor) else x
      rows.append(t.reshape(-1, t.shape[-1]))
    for k in sorted({k for _, _, k in items}):  # one launch per distinct top_k (usually one)
      idx = [i for i, it in enumerate(items) if it[2] == k]
      logits = torch.cat([rows[i].to(self.device, torch.float32) for i in idx]).contiguous()
      temps = self._temps([items[i][1] for i in idx for _ in range(rows[i].shape[0])], self.device)
      tok = K.sample(logits, temps, k, self._seed(self.device))
      self._advance_seed(self.device)
      tok = tok.cpu().numpy().astype(np.int64)
      off = 0
      for i in idx:
        n = rows[i].shape[0]
        out[i] = tok[off:off + n]
        off += n
    return out

  # ------------------------------------------------------------------ engine-driven decode loop
  def continue_locally(self, request_id: str, shard: Shard, token: int, state: dict, emit, fail=None,
                       stop=None) -> bool:
    """Take over a request whose every layer is on this peer: its next steps are queued right after each
    batched forward with the token drawn there (_presample), and `emit(request_id, token) -> finished` is
    called once per token on the event loop -- instead of a chain of Node coroutines (sample, result
    handling, forward_tensor, infer_tensor) per request per token, which at 64 concurrent streams cost more
    host time than the GPU step itself.  `stop(request_id, token) -> bool` predicts emit's answer without
    side effects; with it the next step is queued and launched BEFORE the step's tokens are emitted, so the
    token callbacks (SSE writes of every stream) run while the GPU computes the next step.  Returns False
    when the engine cannot (then the Node forwards the token as usual)."""
    if not (ENGINE_LOOP and PRESAMPLE and self.runner is not None and shard == self.shard
            and shard.is_first_layer() and shard.is_last_layer() and state.get("temperature") is not None):
      return False
    self._loops[request_id] = (emit, fail, stop)
    self._queue.append((request_id, shard, np.asarray([[token]], dtype=np.int64), None, state))
    if not self._draining:
      self._draining = True
      asyncio.create_task(self._drain())
    return True

  async def _loop_next(self, items, results) -> list:
    """Tokens of the engine-loop requests of one step.  Requests whose `stop` predicts they go on are queued
    for the next step at once; returns the (request, token, queued) emissions to make."""
    out = []
    for it, (logits, row) in zip(items, results):  # (step logits [B, V], this request's row)
      rid, shard, _, _, state = it
      cb = self._loops.get(rid)
      if cb is None:
        continue
      hit = self._presampled.pop((logits.data_ptr(), row), None)
      if hit is not None:
        self.stats["presampled"] = self.stats.get("presampled", 0) + 1
        tok = int(hit[2][0])
      else:  # not drawn with the forward (should not happen): draw it now
        tok = int(np.asarray(await self.sample(logits[row:row + 1], _temp_of(state),
                                               int(state.get("top_k") or TOP_K))).reshape(-1)[0])
      self.stats["loop_tokens"] = self.stats.get("loop_tokens", 0) + 1
      queued = False
      if cb[2] is not None:
        try:
          queued = not cb[2](rid, tok)
        except Exception:  # noqa: BLE001 - no prediction: emit first, queue after
          queued = False
        if queued:
          self._queue.append((rid, shard, np.asarray([[tok]], dtype=np.int64), None, state))
      out.append((it, tok, queued))
    return out

  def _emit(self, emissions) -> None:
    """Report the tokens of one step (see _loop_next); reconcile requests the consumer ended differently."""
    for it, tok, queued in emissions:
      rid = it[0]
      cb = self._loops.get(rid)
      if cb is None:
        continue
      try:
        finished = cb[0](rid, tok)
      except Exception:  # noqa: BLE001 - a failing consumer ends its request, not the loop
        finished = True
      if finished:
        self._loops.pop(rid, None)
        if queued:  # still waiting in the queue: drop it (one already cut into a step is skipped by rid)
          self._queue = [q for q in self._queue if not (q[0] == rid and q[3] is None)]
      elif not queued:
        self._queue.append((rid, it[1], np.asarray([[tok]], dtype=np.int64), None, it[4]))

  # ------------------------------------------------------------------ chained engine-loop steps
  def _chainable(self, k: Optional[int] = None) -> bool:
    """The waiting work is engine-loop decode steps only (one token each) sharing one sampler top_k (the
    running chained step's, when given)."""
    if not (CHAIN and self.runner is not None and self._queue):
      return False
    ks = set() if k is None else {k}
    for it in self._queue:
      if it[3] is not None or it[1] != self.shard or self._qlen(it[2]) != 1:
        return False
      ks.add(int(it[4].get("top_k") or TOP_K))
    return len(ks) == 1

  def _plan(self, chain) -> tuple:
    """Next chained step: rows of the running step whose requests go on (by the count-only prediction:
    a request that will have hit its token limit with the running step's token is left out), then queued
    engine-loop requests (host tokens), up to max_batch.  An EOS in the running step is only seen after
    the next step is queued: that request's extra step is discarded."""
    cont = []
    if chain is not None:
      for row, rid in enumerate(chain["rids"]):
        cb = self._loops.get(rid)
        if cb is None:
          continue
        try:
          last = cb[2](rid, -1) if cb[2] is not None else False
        except Exception:  # noqa: BLE001
          last = True
        if not last:
          cont.append((rid, row))
    k = int(chain["states"][0].get("top_k") or TOP_K) if chain is not None and chain["rids"] else None
    room = self.runner.max_batch - len(cont)
    new, rest = [], []
    seen = {rid for rid, _ in cont}
    for it in self._queue:
      ok = (it[3] is None and it[0] in self._loops and it[0] not in seen and self._qlen(it[2]) == 1
            and (k is None or int(it[4].get("top_k") or TOP_K) == k))
      if ok and len(new) < room:
        new.append(it)
        seen.add(it[0])
      elif it[3] is not None or it[0] in self._loops:
        rest.append(it)
    self._queue = rest
    return cont, new

  def _chain_step(self, chain, cont, new):
    """Executor: queue one engine-loop decode step whose inputs are the running step's sampled ids (rows
    `cont`, gathered on the device) and the host tokens of `new`; queue its sampler; then read the running
    step's tokens on the host, which overlaps the new step's GPU work.  Returns (the running step's tokens
    as int64 numpy or None, the new running step or None, requests left out for lack of KV pages).

    KV pressure: when the step's new pages exceed the free pool even after prefix-cache eviction, the
    youngest requests (queued joiners first, then the running rows from the back) give their pages back here
    until the rest fit, and are reported so the event loop ends them ("length") -- instead of the whole step
    failing for every request."""
    t0 = time.perf_counter()
    nxt = None
    victims = []
    try:
      bm = self.runner.bm
      if cont or new:
        need = [bm.blocks_needed(r, 1) for r, _ in cont] + [bm.blocks_needed(it[0], 1) for it in new]
        if sum(need) > bm.num_free:
          if self.prefix_cache is not None:
            self.prefix_cache.evict(sum(need))
          while (cont or new) and sum(need) > bm.num_free:
            v = new.pop()[0] if new else cont.pop()[0]
            need.pop()
            victims.append(v)
            self.runner.free(v)  # its pages (those not shared with a cached prefix) return to the pool now
      if cont or new:
        dev = self.runner.device
        rids = [r for r, _ in cont] + [it[0] for it in new]
        states = [chain["states"][row] for _, row in cont] + [it[4] for it in new]
        parts = []
        if cont:
          rows = [row for _, row in cont]
          if rows == list(range(len(chain["rids"]))):
            parts.append(chain["tok"])
          else:
            idx = torch.tensor(rows, dtype=torch.int64)
            parts.append(chain["tok"].index_select(0, (idx.pin_memory() if dev.type == "cuda" else idx)
                                                   .to(dev, non_blocking=True)))
        if new:
          ids = torch.tensor([int(np.asarray(it[2]).reshape(-1)[0]) for it in new], dtype=torch.int32)
          parts.append((ids.pin_memory() if dev.type == "cuda" else ids).to(dev, non_blocking=True))
        x = parts[0] if len(parts) == 1 else torch.cat(parts)
        pc = self.prefix_cache
        if pc is not None:
          for rid in rids:
            pc.on_decode(rid)
            pc.outgoing_drops(rid)
          need = sum(self.runner.bm.blocks_needed(r, 1) for r in rids)
          if need > self.runner.bm.num_free:
            pc.evict(need)
        if self.trainer is not None and self.trainer.dirty:
          self.trainer.sync_to_inference()
        from ..ops import kernels as K
        ev = STEP_EVENTS and dev.type == "cuda"
        if ev:
          e0 = torch.cuda.Event(enable_timing=True)
          e0.record()
        logits = self.runner.forward(rids, [1] * len(rids), x)
        temps = self._temps([_temp_of(st) for st in states], dev)
        tok = K.sample(logits, temps, int(states[0].get("top_k") or TOP_K), self._seed(dev))
        self._advance_seed(dev)
        nxt = {"rids": rids, "states": states, "tok": tok}
        if dev.type == "cuda":
          # the ids go to the host right behind this step's sampler: a plain .cpu() in the NEXT call would be
          # ordered after the step queued there, i.e. wait for it, and leave the GPU idle between steps
          host = torch.empty(tok.shape, dtype=tok.dtype, pin_memory=True)
          host.copy_(tok, non_blocking=True)
          done = torch.cuda.Event()
          done.record()
          nxt["host"], nxt["done"] = host, done
        if ev:
          e1 = torch.cuda.Event(enable_timing=True)
          e1.record()
          nxt["events"] = (e0, e1)
        self.stats["steps"] += 1
        self.stats["requests"] += len(rids)
        self.stats["chained"] = self.stats.get("chained", 0) + 1
      t1 = time.perf_counter()
      prev = None
      if chain is not None:
        if "done" in chain:
          chain["done"].synchronize()
          prev = chain["host"].numpy().astype(np.int64)
        else:
          prev = chain["tok"].cpu().numpy().astype(np.int64)
      if chain is not None and "events" in chain:  # GPU time of the running step and the idle gap before it
        e0, e1 = chain["events"]
        e1.synchronize()
        self.stats["gpu_step_s"] = self.stats.get("gpu_step_s", 0.0) + e0.elapsed_time(e1) * 1e-3
        last = getattr(self, "_last_end_ev", None)
        if last is not None:
          self.stats["gpu_gap_s"] = self.stats.get("gpu_gap_s", 0.0) + last.elapsed_time(e0) * 1e-3
          self.stats["gpu_gaps"] = self.stats.get("gpu_gaps", 0) + 1
        self._last_end_ev = e1
      self.stats["launch_s"] = self.stats.get("launch_s", 0.0) + t1 - t0  # host prep + graph launch
      self.stats["wait_s"] = self.stats.get("wait_s", 0.0) + time.perf_counter() - t1  # the running step's ids
      return prev, nxt, victims
    finally:
      self.stats["step_s"] = self.stats.get("step_s", 0.0) + time.perf_counter() - t0

  def _emit_chain(self, chain, toks) -> None:
    """Report a finished chained step's tokens.  A request the prediction left out of the next step but
    the consumer did not end goes back to the queue with its host token."""
    nxt_rows = None
    for row, rid in enumerate(chain["rids"]):
      cb = self._loops.get(rid)
      if cb is None:
        continue
      tok = int(toks[row])
      self.stats["loop_tokens"] = self.stats.get("loop_tokens", 0) + 1
      self.stats["chained_tokens"] = self.stats.get("chained_tokens", 0) + 1
      try:
        finished = cb[0](rid, tok)
      except Exception:  # noqa: BLE001 - a failing consumer ends its request, not the loop
        finished = True
      if finished:
        self._loops.pop(rid, None)
        self._queue = [q for q in self._queue if not (q[0] == rid and q[3] is None)]
      else:
        if nxt_rows is None:
          nxt_rows = chain.get("next_rids", set())
        if rid not in nxt_rows:
          self._queue.append((rid, self.shard, np.asarray([[tok]], dtype=np.int64), None, chain["states"][row]))

  def _loop_failed(self, items, err) -> None:
    for it in items:
      cb = self._loops.pop(it[0], None)
      if cb is not None and cb[1] is not None:
        if DEBUG >= 1:
          print(f"[engine] request {it[0]} failed in the decode loop: {err}")
        cb[1](it[0])

  # ------------------------------------------------------------------ prompts with images (LLaVA)
  async def infer_prompt(self, request_id: str, shard: Shard, prompt: str,
                         inference_state: Optional[dict] = None) -> Tuple[object, Optional[dict]]:
    """Prompts may carry `<|xot_image:URL|>` markers (api/chatgpt_api.py keeps the chat's last image that
    way).  A vision model's first shard expands each into its image-token run and keeps the preprocessed
    pixels for the request's prefill; any other model reads the marker as a placeholder text."""
    from ..models.vision import encode_with_images, image_pixels, split_image_marks
    pieces, urls = split_image_marks(prompt)
    if not urls:
      return await super().infer_prompt(request_id, shard, prompt, inference_state)
    await self.ensure_shard(shard)
    c = self.config
    if c.vision is None or not shard.is_first_layer():
      text = "".join(p + ("[image]" if i < len(urls) else "") for i, p in enumerate(pieces))
      return await super().infer_prompt(request_id, shard, text, inference_state)
    ids, urls = encode_with_images(self.tokenizer, c, prompt)
    pixels = await self._run(lambda: image_pixels(c, urls))
    self._images[request_id] = pixels
    return await self.infer_tensor(request_id, shard, np.asarray(ids, dtype=np.int64).reshape(1, -1),
                                   inference_state)

  # ------------------------------------------------------------------ forward (continuously batched)
  async def infer_tensor(self, request_id: str, shard: Shard, input_data,
                         inference_state: Optional[dict] = None) -> Tuple[object, Optional[dict]]:
    """Queue one request's step; concurrent requests on this peer run as ONE batched forward
    (prefill chunks and decode tokens mixed, varlen attention; a pure-decode batch replays the
    HIP graph of its batch bucket).  The reference runs every request on its own, one token at a
    time, through a single global KV cache (sharded_inference_engine.py:230-370)."""
    await self.ensure_shard(shard)
    fut = asyncio.get_running_loop().create_future()
    self._queue.append((request_id, shard, input_data, fut, inference_state or {}))
    if not self._draining:
      self._draining = True
      asyncio.create_task(self._drain())
    return await fut

  @staticmethod
  def _qlen(inp) -> int:
    shape = inp.shape if hasattr(inp, "shape") else np.asarray(inp).shape
    return int(shape[1]) if len(shape) >= 2 else int(np.prod(shape))

  def _take_batch(self) -> list:
    """Next step's requests: up to max_batch of them and MAX_STEP_TOKENS new tokens in all (decode
    tokens and prefill prompts mix; a prompt longer than the budget runs alone, chunked)."""
    cap = self.runner.max_batch if self.runner is not None else 1
    batch, rest, tokens = [], [], 0
    for it in self._queue:
      n = self._qlen(it[2])
      if len(batch) < cap and (not batch or tokens + n <= MAX_STEP_TOKENS):
        batch.append(it)
        tokens += n
      else:
        rest.append(it)
    self._queue = rest
    return batch

  async def _settle(self):
    """Let the requests that are about to queue do so before a step is cut: after a batched step each
    request's next input arrives through a chain of a few tasks (sample -> result handling -> forward),
    and cutting the step at the first arrival would split one decode round into several forward passes,
    each re-reading every weight."""
    prev, stable = -1, 0
    for _ in range(32):
      n = len(self._queue)
      stable = stable + 1 if n == prev else 0
      if stable >= 3:
        return
      prev = n
      await asyncio.sleep(0)

  def _launch(self):
    """Cut the next step from the queue and start it on the executor: (future, items, engine-loop items),
    or None when nothing in the cut can run."""
    batch = self._take_batch()
    ok = []
    for it in batch:
      if it[3] is None and it[0] not in self._loops:
        continue  # an engine-loop request that ended after its step was queued
      if it[1] != self.shard:
        err = RuntimeError(f"shard {it[1]} is not loaded on this peer (have {self.shard})")
        if it[3] is None:
          self._loop_failed([it], err)
        elif not it[3].done():
          it[3].set_exception(err)
        continue
      ok.append(it)
    if not ok:
      return None
    fut = asyncio.get_running_loop().run_in_executor(self.executor, self._infer_batch,
                                                     [(it[0], it[2], it[4], it[3] is None) for it in ok])
    return fut, ok, [it for it in ok if it[3] is None]

  async def _drain(self):
    """Step loop.  While only engine-loop requests are waiting, step N+1 is launched before step N's
    tokens are emitted (host work overlaps the GPU); a step that carried Node-path requests first lets
    their follow-ups queue (_settle), so one decode round stays one forward pass."""
    pending = None
    chain = None  # chained engine-loop step running on the device (see _chain_step)
    loop = asyncio.get_running_loop()
    try:
      while self._queue or pending is not None or chain is not None:
        if pending is None and (chain is not None or self._chainable()):
          k = int(chain["states"][0].get("top_k") or TOP_K) if chain is not None else None
          if not self._queue or self._chainable(k):
            cont, new = self._plan(chain)
            if chain is None and not new:
              continue
          else:  # other work is waiting (Node-path steps, another top_k): finish the chained step first
            cont, new = [], []
          running = chain
          try:
            toks, chain, victims = await loop.run_in_executor(self.executor, self._chain_step, running, cont, new)
          except Exception as e:  # noqa: BLE001
            self._loop_failed([(r,) for r in (running["rids"] if running else [])] + new, e)
            chain = None
            continue
          if running is not None:
            # a victim gets the running step's token, then ends (not re-queued)
            running["next_rids"] = (set(chain["rids"]) if chain is not None else set()) | set(victims)
            self._emit_chain(running, toks)
          if victims:
            self.stats["kv_evicted_requests"] = self.stats.get("kv_evicted_requests", 0) + len(victims)
            self._queue = [q for q in self._queue if not (q[3] is None and q[0] in victims)]
            self._loop_failed([(r,) for r in victims], RuntimeError("KV cache full"))
          continue
        if pending is None:
          await self._settle()
          pending = self._launch()
          if pending is None:
            continue
        fut, ok, looped = pending
        pending = None
        try:
          results = await fut
        except Exception as e:  # noqa: BLE001 - delivered to every waiter of the batch
          for it in ok:
            if it[3] is not None and not it[3].done():
              it[3].set_exception(e)
          self._loop_failed(looped, e)
          continue
        node_path = False
        for it, r in zip(ok, results):
          if it[3] is not None:
            node_path = True
            if not it[3].done():
              it[3].set_result(r)
        emissions = []
        if looped:
          emissions = await self._loop_next(looped, [r for it, r in zip(ok, results) if it[3] is None])
        if self._queue and not node_path and not self._chainable():
          pending = self._launch()
        self._emit(emissions)
    finally:
      self._draining = False
      if chain is not None:
        self._loop_failed([(r,) for r in chain["rids"]], RuntimeError("engine step loop stopped"))
      if pending is not None:  # left abnormally with a step in flight: its waiters get an error, not a hang
        err = RuntimeError("engine step loop stopped")
        for it in pending[1]:
          if it[3] is not None and not it[3].done():
            it[3].set_exception(err)
        self._loop_failed(pending[2], err)

  def _infer_batch(self, items):
    t0 = time.perf_counter()
    try:
      return self._infer_batch_impl(items)
    finally:
      self.stats["step_s"] = self.stats.get("step_s", 0.0) + time.perf_counter() - t0

  def _infer_batch_impl(self, items):
    self.stats["steps"] += 1
    self.stats["requests"] += len(items)
    if self.trainer is not None and self.trainer.dirty:
      self.trainer.sync_to_inference()  # serve the weights training just produced
    rids, qlens, xs, pc_ops = [], [], [], []
    pc = self.prefix_cache
    for rid, inp, *rest in items:
      state = (rest[0] if rest else None) or {}
      ops = None
      if (inp.dim() if isinstance(inp, torch.Tensor) else np.ndim(inp)) == 3:  # hidden [1, L, D]
        from .prefix_cache import apply_ops
        apply_ops(self.runner.bm, rid, state.get("pc"))  # the first shard's prefix-cache operations
        x = inp if isinstance(inp, torch.Tensor) else torch.as_tensor(np.asarray(inp))
        L = x.shape[1]
        xs.append(x.reshape(L, x.shape[2]).to(torch.bfloat16))
      else:  # token ids [1, L]: numpy on the host (no per-request tensor ops; one tensor for the step)
        ids = (inp.detach().cpu().numpy() if isinstance(inp, torch.Tensor) else np.asarray(inp)).reshape(-1)
        if pc is not None and state.get("kv_min"):
          # the smallest KV pool on the ring (reported by every downstream shard): downstream shards never
          # evict holders themselves, so the cap must fit the smallest pool, not just this one
          pc.cap = min(pc.cap, int(int(state["kv_min"]) * PREFIX_CACHE_FRAC))
        if pc is not None and rid not in self._images:
          ops = {}
          if ids.size > 1 and not self.runner.has(rid):
            n, eid = pc.on_prompt(rid, ids.tolist())
            if n:
              ids = ids[n:]
              ops["fork"] = [eid, n]
          elif ids.size == 1 and self.runner.has(rid):
            save = pc.on_decode(rid)
            if save is not None:
              ops["save"] = save
          drops = pc.outgoing_drops(rid)
          if drops:
            ops["drop"] = drops
        xs.append(ids)
        L = int(ids.size)
      rids.append(rid)
      qlens.append(L)
      pc_ops.append(ops or None)
    if pc is not None:
      need = sum(self.runner.bm.blocks_needed(r, q) for r, q in zip(rids, qlens))
      if need > self.runner.bm.num_free:
        pc.evict(need)
    image_embeds = None
    if self._images and self.shard.is_first_layer():
      feats = [self.runner.image_features(self._images.pop(rid)) for rid in rids if rid in self._images]
      image_embeds = torch.cat(feats) if feats else None
    t_prep = time.perf_counter()
    try:
      if all(isinstance(t, np.ndarray) for t in xs):
        x = torch.from_numpy(np.concatenate(xs).astype(np.int32, copy=False))
      else:
        x = torch.cat([torch.from_numpy(t.astype(np.int32)) if isinstance(t, np.ndarray) else t for t in xs])
      if sum(qlens) > MAX_STEP_TOKENS and len(rids) == 1:
        out = self._forward_chunked(rids[0], x, image_embeds)
      else:
        out = (self.runner.forward(rids, qlens, x) if image_embeds is None
               else self.runner.forward(rids, qlens, x, image_embeds=image_embeds))
    except torch.cuda.OutOfMemoryError:
      self.clear_model()
      raise
    res = []
    if self.shard.is_last_layer():
      # [B, V] fp32 logits of each request's last token; they stay on the device for the sampler.  A copy:
      # a decode step's logits live in its HIP graph's static buffer, which the next step of the same batch
      # bucket overwrites, possibly before every request of this step has sampled
      out = out.clone()
      t_launched = time.perf_counter()
      self._presample(out, [it[2] if len(it) > 2 else {} for it in items])
      st = self.stats
      st["launch_s"] = st.get("launch_s", 0.0) + t_launched - t_prep  # host prep + kernel / graph launch
      st["wait_s"] = st.get("wait_s", 0.0) + time.perf_counter() - t_launched  # sampler + the token copy
      kv_min = self.runner.bm.num_blocks
      for i, (rid, it) in enumerate(zip(rids, items)):
        if len(it) > 3 and it[3]:  # engine-loop request: (logits, row) -- no view, no state to ship
          res.append((out, i))
        else:
          st = {"n_past": self.runner.num_tokens(rid)}
          if not self.shard.is_first_layer():  # smallest KV pool of the ring, for the first shard's cache cap
            prev = ((it[2] if len(it) > 2 else None) or {}).get("kv_min")
            st["kv_min"] = min(kv_min, int(prev)) if prev else kv_min
          res.append((out[i:i + 1], st))
      return res
    off = 0
    outc = out.cpu()
    kv_min = self.runner.bm.num_blocks
    for (rid, _, *rest), L, ops in zip(items, qlens, pc_ops):
      st = {"n_past": self.runner.num_tokens(rid)}
      if self.shard.is_first_layer():
        st["pc"] = ops  # replaces the previous step's operations in the state that travels the ring
      else:
        prev = ((rest[0] if rest else None) or {}).get("kv_min")
        st["kv_min"] = min(kv_min, int(prev)) if prev else kv_min
      res.append((outc[off:off + L].reshape(1, L, -1), st))
      off += L
    return res

  def _forward_chunked(self, rid: str, x: torch.Tensor, image_embeds: Optional[torch.Tensor]):
    """Chunked prefill of one long prompt: MAX_STEP_TOKENS-token pieces appended to its KV in turn.
    Returns the last piece's logits (last shard) or every piece's hidden states (other shards)."""
    outs, used = [], 0
    img_id = self.config.image_token_id
    for lo in range(0, x.shape[0], MAX_STEP_TOKENS):
      xc = x[lo:lo + MAX_STEP_TOKENS]
      emb = None
      if image_embeds is not None:
        n = int((xc == img_id).sum()) if xc.dim() == 1 else 0
        emb = image_embeds[used:used + n] if n else None
        used += n
      y = (self.runner.forward([rid], [xc.shape[0]], xc) if emb is None
           else self.runner.forward([rid], [xc.shape[0]], xc, image_embeds=emb))
      outs.append(y if self.shard.is_last_layer() else y.clone())
    return outs[-1] if self.shard.is_last_layer() else torch.cat(outs)

  async def finish_request(self, request_id: str, ok: bool = True) -> None:
    self._images.pop(request_id, None)
    self._loops.pop(request_id, None)
    if self.runner is not None:
      pc = self.prefix_cache

      def fin():
        if pc is not None:
          pc.on_finish(request_id, ok=ok)
        self.runner.free(request_id)
      await self._run(fin)

  # ------------------------------------------------------------------ shard lifecycle
  def _model_dir(self, shard: Shard) -> Optional[Path]:
    repo = registry.get_repo(shard.model_id, "ShardedInferenceEngine")
    if repo is None:
      return None
    from ..helpers import xot_home
    p = xot_home() / "downloads" / repo.replace("/", "--")
    return p if (p / "config.json").exists() else None

  async def ensure_shard(self, shard: Shard):
    if self.shard == shard and self.runner is not None:
      return
    async with self._lock:
      if self.shard == shard and self.runner is not None:
        return
      model_dir = None
      if self.shard_downloader is not None and shard.model_id not in registry.SYNTHETIC:
        try:
          model_dir = await self.shard_downloader.ensure_shard(shard, "ShardedInferenceEngine")
        except Exception as e:
          if DEBUG >= 1:
            print(f"download of {shard.model_id} unavailable ({e}); using synthetic weights")
      model_dir = Path(model_dir) if model_dir else self._model_dir(shard)
      await self._run(self._build, shard, model_dir)

  def _build(self, shard: Shard, model_dir: Optional[Path]):
    from ..models.weights import load_hf_weights
    from ..runtime.runner import ShardRunner
    self.clear_model()
    if model_dir is not None and (model_dir / "config.json").exists():
      cfg = load_config(model_dir)
      registry.validate_layers(shard.model_id, cfg.num_layers)
    else:
      cfg = preset(shard.model_id)
    if cfg.num_layers != shard.n_layers:
      cfg = cfg.with_layers(shard.n_layers)
    weights = None
    if model_dir is not None and any(model_dir.glob("*.safetensors")):
      weights = load_hf_weights(model_dir, cfg, shard, self.device)
    elif DEBUG >= 1:
      print(f"[engine] {shard.model_id}: no local weights, random-init {cfg.model_type} shard {shard}")
    max_ctx = int(os.environ.get("XOT_MAX_CTX", 8192 if self.device.type == "cuda" else 2048))
    max_ctx = min(max_ctx, cfg.max_position_embeddings)
    self.runner = ShardRunner(cfg, shard, self.device, weights=weights, max_batch=int(os.environ.get("XOT_MAX_BATCH", 64)),
                              max_ctx=max_ctx, seed=0)
    self.config = cfg
    self.model_path = model_dir
    self.prefix_cache = None
    longrope = (cfg.rope_scaling or {}).get("rope_type") == "longrope"  # the prefix's rotation depends on the total length
    if PREFIX_CACHE and shard.is_first_layer() and not longrope:
      from .prefix_cache import PrefixCache
      self.prefix_cache = PrefixCache(self.runner.bm, int(self.runner.bm.num_blocks * PREFIX_CACHE_FRAC),
                                      single_shard=shard.is_last_layer())
    self.tokenizer = _resolve_tokenizer(model_dir if model_dir is not None else
                                        (registry.get_repo(shard.model_id, "ShardedInferenceEngine") or "byte"),
                                        cfg.vocab_size)
    self.shard = shard

  def clear_model(self):
    self.runner = None
    self.shard = None
    if self.device.type == "cuda":
      torch.cuda.empty_cache()

  @property
  def eos_token_ids(self):
    ids = set(self.config.eos_token_ids) if self.config else set()
    tid = getattr(self.tokenizer, "eos_token_id", None)
    if tid is not None:
      ids.add(int(tid))
    return ids

  # ------------------------------------------------------------------ checkpoints / training
  async def load_checkpoint(self, shard: Shard, path: str):
    from ..train.checkpoint import load_shard_checkpoint
    await self.ensure_shard(shard)
    await self._run(load_shard_checkpoint, self, shard, path)

  async def save_checkpoint(self, shard: Shard, path: str):
    from ..train.checkpoint import save_shard_checkpoint
    await self.ensure_shard(shard)
    await self._run(save_shard_checkpoint, self, shard, path)

  def _get_trainer(self):
    from ..train.trainer import ShardTrainer
    if self.trainer is None or self.trainer.shard != self.shard:
      self.trainer = ShardTrainer(self.runner.weights, self.device, lr=self.lr)
    return self.trainer

  async def train(self, request_id, shard, example, target, length, train=True, loss="length_masked_ce"):
    await self.ensure_shard(shard)
    return await self._run(lambda: self._get_trainer().step(request_id, example, target, length, train=train,
                                                            loss=loss))

  async def train_forward(self, request_id, shard, example):
    """Forward of a non-last pipeline stage for training (no KV cache): the activation to send on."""
    await self.ensure_shard(shard)
    return await self._run(lambda: self._get_trainer().train_forward(example))

  async def eval_forward(self, request_id, shard, example):
    return await self.train_forward(request_id, shard, example)

  async def evaluate(self, request_id, shard, example, target, length, loss="length_masked_ce"):
    await self.ensure_shard(shard)
    return await self._run(lambda: self._get_trainer().step(request_id, example, target, length, train=False,
                                                            evaluate=True))

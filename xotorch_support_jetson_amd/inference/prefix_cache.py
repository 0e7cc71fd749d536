"""Prompt-prefix KV reuse across requests, consistent over a ring of shards.

Chat clients resend the whole conversation every turn (the reference's tinychat, index.js, posts the full
message history), so without reuse every turn re-prefills everything said so far.  Here the KV pages of a
served prompt stay in the shard's pool after the request ends, held by a refcounted holder sequence
(`pc:<id>`, BlockManager.fork shares whole 64-token pages), and a later prompt that starts with the same
pages forks them and prefills only the rest.

Only the first shard sees token ids, so it owns the policy (hashing, lookup, LRU eviction); every other
shard applies the operations it attaches to a request's inference state, in the order that request's steps
reach it:
  save  [id, ntok]  on a request's first decode step: fork its first ntok prompt tokens into holder pc:id
  fork  [id, ntok]  on a prefill: fork holder pc:id into the new request; its input covers tokens ntok..
  drop  [ids]       free holders
The protocol never lets an operation overtake the one it depends on:
  * an entry is used for a fork only once it is confirmed: the saving request came back to the first
    shard for another step (so every shard applied the save), or finished normally (likewise; a request
    that failed part-way drops its unconfirmed entry instead);
  * an entry is dropped only when no fork of it is pending: each fork is confirmed by the forking
    request's next step or its end;
  * drop ids ride on every outgoing state until a request that carried them comes back.
Downstream shards never evict on their own; the first shard caps the cached pages at a fraction of its
pool (pools are sized alike: the ring partitioner gives layers in proportion to memory).
"""
from __future__ import annotations

import hashlib
from collections import OrderedDict
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

PAGE = 64


def holder(eid: int) -> str:
  return f"pc:{eid}"


def page_hashes(tokens: Sequence[int], n_pages: int) -> List[bytes]:
  """Chain hashes of the first n_pages full pages: h_i covers tokens [0, 64 (i + 1))."""
  out, h = [], b""
  arr = np.asarray(tokens[:n_pages * PAGE], dtype=np.int64)
  for i in range(n_pages):
    h = hashlib.blake2b(h + arr[i * PAGE:(i + 1) * PAGE].tobytes(), digest_size=16).digest()
    out.append(h)
  return out


@dataclass
class Entry:
  eid: int
  hashes: List[bytes]
  confirmed: bool = False
  pending: int = 0  # forks not yet confirmed

  @property
  def pages(self) -> int:
    return len(self.hashes)


@dataclass
class ReqInfo:
  hashes: List[bytes]  # full-page chain hashes of the prompt
  fork: Optional[int] = None  # entry forked at prefill, until confirmed
  saved: Optional[int] = None  # entry this request saved, until confirmed
  steps: int = 0  # decode steps seen on the first shard
  drops: Tuple[int, ...] = ()  # drop ids its last outgoing state carried


class PrefixCache:
  """First-shard policy.  All methods run on the engine's executor thread (the BlockManager owner)."""

  def __init__(self, bm, cap_pages: int, single_shard: bool):
    self.bm = bm
    self.cap = max(0, int(cap_pages))
    self.single = single_shard  # one shard holds every layer: nothing to confirm
    self.entries: "OrderedDict[int, Entry]" = OrderedDict()  # LRU order
    self.by_hash: Dict[bytes, Tuple[int, int]] = {}  # chain hash -> (entry id, pages)
    self.reqs: Dict[str, ReqInfo] = {}
    self.drop_q: Dict[int, None] = {}
    self.next_id = 0
    self.stats = {"hit_tokens": 0, "prompts": 0, "saved": 0, "evicted": 0}

  # ------------------------------------------------------------------ bookkeeping
  def cached_pages(self) -> int:
    return sum(e.pages for e in self.entries.values())

  def _drop(self, e: Entry) -> None:
    self.entries.pop(e.eid, None)
    for i, h in enumerate(e.hashes):
      if self.by_hash.get(h, (None,))[0] == e.eid:
        del self.by_hash[h]
    self.bm.free(holder(e.eid))
    if not self.single:
      self.drop_q[e.eid] = None
    self.stats["evicted"] += 1

  def evict(self, need_pages: int) -> None:
    """Free least-recently-used entries with no pending fork until need_pages pages are free."""
    for e in list(self.entries.values()):
      if self.bm.num_free >= need_pages:
        return
      if e.pending == 0 and (e.confirmed or self.single):
        self._drop(e)

  def _fit(self, pages: int) -> bool:
    """Room under the cap for an entry of `pages` pages (evicting LRU entries)."""
    if pages > self.cap:
      return False
    for e in list(self.entries.values()):
      if self.cached_pages() + pages <= self.cap:
        break
      if e.pending == 0 and (e.confirmed or self.single):
        self._drop(e)
    return self.cached_pages() + pages <= self.cap

  # ------------------------------------------------------------------ steps
  def on_prompt(self, rid: str, tokens: Sequence[int]) -> Tuple[int, Optional[int]]:
    """A new prompt on the first shard: fork the longest cached prefix (whole pages, at least one token
    left to run) into rid.  Returns (prompt tokens reused, entry id)."""
    n = len(tokens)
    hashes = page_hashes(tokens, n // PAGE)
    info = ReqInfo(hashes)
    self.reqs[rid] = info
    self.stats["prompts"] += 1
    usable = (n - 1) // PAGE
    best = None
    for i in range(min(usable, len(hashes)) - 1, -1, -1):
      hit = self.by_hash.get(hashes[i])
      if hit is None:
        continue
      e = self.entries.get(hit[0])
      if e is not None and (e.confirmed or self.single) and e.hashes[i] == hashes[i]:
        best = (e, i + 1)
        break
    if best is None or self.bm.has(rid):
      return 0, None
    e, pages = best
    self.bm.fork(holder(e.eid), rid, pages * PAGE)
    self.entries.move_to_end(e.eid)
    if not self.single:
      e.pending += 1
      info.fork = e.eid
    self.stats["hit_tokens"] += pages * PAGE
    return pages * PAGE, e.eid

  def on_decode(self, rid: str) -> Optional[list]:
    """A decode step of rid reached the first shard (its previous step went round the whole ring).
    Confirms what that request left pending; on its first decode step saves its prompt pages.
    Returns the save op [id, ntok] or None."""
    info = self.reqs.get(rid)
    if info is None:
      return None
    info.steps += 1
    self._confirm(info)
    for d in info.drops:  # the drops its last state carried reached every shard
      self.drop_q.pop(d, None)
    info.drops = ()
    if info.steps != 1 or not info.hashes:
      return None
    pages = len(info.hashes)
    known = self.by_hash.get(info.hashes[-1])
    if known is not None and known[0] in self.entries:
      self.entries.move_to_end(known[0])
      return None
    if not self._fit(pages) or self.bm.num_tokens(rid) < pages * PAGE:
      return None
    eid = self.next_id
    self.next_id += 1
    self.bm.fork(rid, holder(eid), pages * PAGE)
    e = Entry(eid, list(info.hashes), confirmed=self.single)
    self.entries[eid] = e
    for i, h in enumerate(info.hashes):  # a prefix another live entry already serves keeps pointing there
      cur = self.by_hash.get(h)
      if cur is None or cur[0] not in self.entries:
        self.by_hash[h] = (eid, i + 1)
    if not self.single:
      info.saved = eid
    self.stats["saved"] += 1
    return [eid, pages * PAGE]

  def _confirm(self, info: ReqInfo) -> None:
    if info.fork is not None:
      e = self.entries.get(info.fork)
      if e is not None:
        e.pending = max(0, e.pending - 1)
      info.fork = None
    if info.saved is not None:
      e = self.entries.get(info.saved)
      if e is not None:
        e.confirmed = True
      info.saved = None

  def outgoing_drops(self, rid: str) -> list:
    """Drop ids to attach to rid's outgoing state (repeated until a carrier comes back)."""
    ids = list(self.drop_q)
    info = self.reqs.get(rid)
    if info is not None and ids:
      info.drops = tuple(ids)
    return ids

  def on_finish(self, rid: str, ok: bool = True) -> None:
    """ok: the request ended normally (announced by the last shard), so every step it sent went through
    every shard.  A failed or aborted request gives no such guarantee: the save it carried may never have
    reached the downstream shards, so its unconfirmed entry is dropped instead of confirmed (a later fork
    of it would find no holder there), and the drops it carried stay queued for the next carrier."""
    info = self.reqs.pop(rid, None)
    if info is None:
      return
    if ok:
      self._confirm(info)
      for d in info.drops:
        self.drop_q.pop(d, None)
      return
    if info.fork is not None:  # nothing else can confirm this fork any more
      e = self.entries.get(info.fork)
      if e is not None:
        e.pending = max(0, e.pending - 1)
      info.fork = None
    if info.saved is not None:
      e = self.entries.get(info.saved)
      if e is not None and not e.confirmed:
        self._drop(e)  # frees the holder here; downstream holders (if any) go with the queued drop
      info.saved = None


def apply_ops(bm, rid: str, ops: Optional[dict]) -> None:
  """Downstream shard: apply the first shard's prefix-cache operations for this step of rid."""
  if not ops:
    return
  for eid in ops.get("drop") or ():
    bm.free(holder(int(eid)))
  save = ops.get("save")
  if save is not None:
    eid, ntok = int(save[0]), int(save[1])
    if not bm.has(holder(eid)) and bm.has(rid) and bm.num_tokens(rid) >= ntok:
      bm.fork(rid, holder(eid), ntok)
  fork = ops.get("fork")
  if fork is not None:
    eid, ntok = int(fork[0]), int(fork[1])
    if not bm.has(holder(eid)):
      raise RuntimeError(f"prefix cache: holder {holder(eid)} missing on this shard (request {rid})")
    if not bm.has(rid):
      bm.fork(holder(eid), rid, ntok)

"""Pure-Python twin of the native BlockManager (csrc/runtime/block_manager.cpp).

Used only where the C++ runtime is not built, and by the tests as an executable specification the
native implementation is checked against.
"""
from __future__ import annotations

from typing import Dict, List


class BlockManager:
  def __init__(self, num_blocks: int, block_size: int = 64):
    if num_blocks <= 0 or block_size <= 0:
      raise ValueError("num_blocks and block_size must be > 0")
    self.block_size = block_size
    self.num_blocks = num_blocks
    self._ref = [0] * num_blocks
    self._free: List[int] = list(range(num_blocks - 1, -1, -1))
    self._seqs: Dict[str, list] = {}  # rid -> [blocks, ntok]

  @property
  def num_free(self) -> int:
    return len(self._free)

  @property
  def num_sequences(self) -> int:
    return len(self._seqs)

  def has(self, rid: str) -> bool:
    return rid in self._seqs

  def num_tokens(self, rid: str) -> int:
    return self._seqs[rid][1]

  def blocks_needed(self, rid: str, extra: int) -> int:
    blocks, ntok = self._seqs.get(rid, ([], 0))
    need = -(-(ntok + extra) // self.block_size)
    return max(0, need - len(blocks))

  def can_append(self, rid: str, extra: int) -> bool:
    return self.blocks_needed(rid, extra) <= self.num_free

  def append(self, rid: str, n: int) -> List[int]:
    if n < 0:
      raise ValueError("append: n < 0")
    need = self.blocks_needed(rid, n)
    if need > self.num_free:
      raise RuntimeError(f"KV cache exhausted: need {need} pages, {self.num_free} free")
    s = self._seqs.setdefault(rid, [[], 0])
    for _ in range(need):
      b = self._free.pop()
      self._ref[b] = 1
      s[0].append(b)
    out = [s[0][t // self.block_size] * self.block_size + t % self.block_size for t in range(s[1], s[1] + n)]
    s[1] += n
    return out

  def truncate(self, rid: str, new_len: int) -> None:
    s = self._seqs[rid]
    if new_len < 0 or new_len > s[1]:
      raise ValueError("truncate: bad length")
    s[1] = new_len
    keep = -(-new_len // self.block_size)
    while len(s[0]) > keep:
      self._release(s[0].pop())

  def free(self, rid: str) -> None:
    s = self._seqs.pop(rid, None)
    if s:
      for b in s[0]:
        self._release(b)

  def fork(self, src: str, dst: str, ntok: int) -> None:
    if dst in self._seqs:
      raise ValueError("fork: destination exists")
    blocks, have = self._seqs[src]
    ntok = min(ntok, have) // self.block_size * self.block_size
    nb = ntok // self.block_size
    for b in blocks[:nb]:
      self._ref[b] += 1
    self._seqs[dst] = [list(blocks[:nb]), ntok]

  def block_table(self, rid: str) -> List[int]:
    return list(self._seqs[rid][0])

  def fill_batch(self, rids, tables, ctx_lens) -> None:
    width = tables.shape[1]
    for i, rid in enumerate(rids):
      blocks, ntok = self._seqs[rid]
      if len(blocks) > width:
        raise ValueError("fill_batch: block table too narrow")
      tables[i, :] = 0
      tables[i, :len(blocks)] = blocks
      ctx_lens[i] = ntok

  def _release(self, b: int) -> None:
    self._ref[b] -= 1
    if self._ref[b] == 0:
      self._free.append(b)

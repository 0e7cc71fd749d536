"""Device weight layouts.

`shuffle_for_stream`: permutes an nn.Linear weight [N, K] (bf16) into the tile order consumed by the
GEMM kernels (gemm_stream with wshuf=True, gemm_big): tiles of 16 rows x 128 k laid out
[N/16][K/128][s][lane][8] where lane = 16*g + c holds row 16*nt + c, k = 128*kc + 32*s + 8*g .. +8,
i.e. block s is exactly the MFMA 16x16x32 B-operand fragment set of k [32s, 32s+32).  One
wave-instruction (64 lanes x 16 B) then reads 1 KB of contiguous memory, instead of sixteen 64-byte row
pieces, and a 64-deep k stage of a 16-row group is 2 KB of contiguous memory (one LDS-DMA copy).
The logical shape stays [N, K]; only the storage order changes.
"""
from __future__ import annotations

import torch


def can_shuffle(w: torch.Tensor) -> bool:
  # tiles of 16 rows x 128 k (the stream GEMM takes any whole number of 128-wide k-chunks per workgroup)
  return w.dim() == 2 and w.shape[0] % 64 == 0 and w.shape[1] % 128 == 0


def shuffle_for_stream(w: torch.Tensor) -> torch.Tensor:
  N, K = w.shape
  v = w.reshape(N // 16, 16, K // 128, 4, 4, 8)  # nt, c, kc, s, g, e
  return v.permute(0, 2, 3, 4, 1, 5).contiguous().reshape(N, K)


def unshuffle_from_stream(ws: torch.Tensor) -> torch.Tensor:
  N, K = ws.shape
  v = ws.reshape(N // 16, K // 128, 4, 4, 16, 8)  # nt, kc, s, g, c, e
  return v.permute(0, 4, 1, 2, 3, 5).contiguous().reshape(N, K)

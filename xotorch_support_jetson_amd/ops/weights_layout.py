"""Device weight layouts.

`shuffle_for_stream`: permutes an nn.Linear weight [N, K] (bf16) into the tile order consumed by the
GEMM kernels (gemm_stream with wshuf=True, gemm_big): tiles of 16 rows x 128 k laid out
[N/16][K/128][s][lane][8] where lane = 16*g + c holds row 16*nt + c, k = 128*kc + 32*s + 8*g .. +8,
i.e. block s is exactly the MFMA 16x16x32 B-operand fragment set of k [32s, 32s+32).  One
wave-instruction (64 lanes x 16 B) then reads 1 KB of contiguous memory, instead of sixteen 64-byte row
pieces, and a 64-deep k stage of a 16-row group is 2 KB of contiguous memory (one LDS-DMA copy).
The logical shape stays [N, K]; only the storage order changes.

`shuffle_for_stream8`: the weight-only FP8 variant (OCP e4m3 bytes + one fp32 scale per output row,
`quantize_fp8_rows`): tiles of 16 rows x 128 k laid out [N/16][K/128][2][lane][16 B], lane (g, c)'s 16
bytes in half h holding row c, k 64h + 8g .. +8 and 64h + 32 + 8g .. +8 -- two MFMA k-steps per 1 KB wave
load (gemm_stream with W8, csrc/gemm.hip).
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


E4M3_MAX = 448.0


def quantize_fp8_rows(w: torch.Tensor):
  """[N, K] -> (e4m3 bits as uint8 [N, K], fp32 scale [N]) with w ~= q * scale[:, None] (row absmax -> 448)."""
  wf = w.float()
  scale = (wf.abs().amax(1) / E4M3_MAX).clamp_min(1e-12)
  q = (wf / scale[:, None]).clamp(-E4M3_MAX, E4M3_MAX).to(torch.float8_e4m3fn)
  return q.view(torch.uint8), scale


def shuffle_for_stream8(q: torch.Tensor) -> torch.Tensor:
  N, K = q.shape
  v = q.reshape(N // 16, 16, K // 128, 2, 2, 4, 8)  # nt, c, kc, s', h, g, e  (k = 128kc + 64s' + 32h + 8g + e)
  return v.permute(0, 2, 3, 5, 1, 4, 6).contiguous().reshape(N, K)


def unshuffle_from_stream8(qs: torch.Tensor) -> torch.Tensor:
  N, K = qs.shape
  v = qs.reshape(N // 16, K // 128, 2, 4, 16, 2, 8)  # nt, kc, s', g, c, h, e
  return v.permute(0, 4, 1, 2, 5, 3, 6).contiguous().reshape(N, K)


def dequant_stream8_to_stream(qs: torch.Tensor, scale: torch.Tensor) -> torch.Tensor:
  """bf16 copy of a shuffled FP8 weight directly in the bf16 shuffled layout (no row-major round trip):
  the 16 bytes of lane (g, c) in half h hold k 64h + 8g and 64h + 32 + 8g, which are lane (g, c) of the
  bf16 blocks s = 2h and 2h + 1."""
  N, K = qs.shape
  q = qs.view(torch.float8_e4m3fn).view(N // 16, K // 128, 2, 64, 2, 8).float()  # nt, kc, h, lane, part, e
  sc = scale.float().view(N // 16, 1, 1, 1, 16).expand(N // 16, 1, 1, 4, 16).reshape(N // 16, 1, 1, 64, 1, 1)
  return (q * sc).to(torch.bfloat16).permute(0, 1, 2, 4, 3, 5).reshape(N, K)


def dequant_stream8(qs: torch.Tensor, scale: torch.Tensor, dtype=torch.bfloat16) -> torch.Tensor:
  """Row-major [N, K] `dtype` copy of a shuffled FP8 weight."""
  q = unshuffle_from_stream8(qs).view(torch.float8_e4m3fn)
  return (q.float() * scale.float()[:, None]).to(dtype)

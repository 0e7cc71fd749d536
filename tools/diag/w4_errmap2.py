#!/usr/bin/env python3
"""Debug: the four-wave tile's SiLU epilogue (natural weight rows, no DMA swizzle) vs the permuted-row epilogues."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from xotorch_support_jetson_amd.ops._ext import require  # noqa: E402
from xotorch_support_jetson_amd.ops.weights_layout import shuffle_for_stream  # noqa: E402

C = require()
g = torch.Generator().manual_seed(0)
M, N, Kd = 256, 256, 128
x = torch.randint(-3, 4, (M, Kd), generator=g).to(torch.bfloat16).cuda()
w = torch.randint(-3, 4, (N, Kd), generator=g).to(torch.bfloat16).cuda()
full = x.float() @ w.float().t()
f = full.view(M, N // 32, 2, 16)
ref = (torch.nn.functional.silu(f[:, :, 0]) * f[:, :, 1]).reshape(M, N // 2)
y = torch.zeros(M, N // 2, device="cuda", dtype=torch.float32)
C.gemm_big(x, shuffle_for_stream(w), y, None, None, None, 2, 4256, 1)
err = ((y - ref).abs() / (ref.abs() + 1)).max().item()
print("silu f32 max rel err", err, "wrong", int(((y - ref).abs() > 1e-3 * (ref.abs() + 1)).sum()))
# slab path (natural / permuted column order inside the kernel, reduced by the split-K reduce kernel)
for epi in (0, 2):
  ws = torch.empty(2 * M * N, device="cuda", dtype=torch.float32)
  yy = torch.zeros(M, N // 2 if epi == 2 else N, device="cuda", dtype=torch.float32)
  C.gemm_big(x, shuffle_for_stream(w), yy, None, None, ws, epi, 4256, 2)
  want = ref if epi == 2 else full
  print("split 2 epi", epi, "wrong", int(((yy - want).abs() > 1e-3 * (want.abs() + 1)).sum()))

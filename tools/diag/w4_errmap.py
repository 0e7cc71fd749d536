#!/usr/bin/env python3
"""Debug: where the four-wave GEMM tile (code 4256) differs from the reference -- (row, col) classes of the wrong
elements for a few small shapes (integer operands: exact products)."""
import os
import sys
from collections import Counter

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from xotorch_support_jetson_amd.ops._ext import require  # noqa: E402
from xotorch_support_jetson_amd.ops.weights_layout import shuffle_for_stream  # noqa: E402

C = require()
g = torch.Generator().manual_seed(0)
for M, N, Kd in [(256, 256, 128), (256, 256, 256), (256, 256, 1024), (256, 1024, 1280)]:
  x = torch.randint(-3, 4, (M, Kd), generator=g).to(torch.bfloat16).cuda()
  w = torch.randint(-3, 4, (N, Kd), generator=g).to(torch.bfloat16).cuda()
  ref = x.float() @ w.float().t()
  y = torch.zeros(M, N, device="cuda", dtype=torch.float32)
  C.gemm_big(x, shuffle_for_stream(w), y, None, None, None, 0, 4256, 1)
  bad = (y != ref).nonzero().tolist()
  print(f"M {M} N {N} K {Kd}: {len(bad)} wrong of {M * N}")
  if bad:
    cls = Counter(((r % 256) // 128, (c % 256) // 128, (r % 16), (c % 128) // 32, (c % 32) // 8, c % 8) for r, c in bad)
    print("  (wm, wn, row%16, J, g, e) most common:", cls.most_common(12))
    rows = Counter(r % 256 for r, c in bad)
    cols = Counter(c % 256 for r, c in bad)
    print("  rows:", sorted(rows)[:40])
    print("  cols:", sorted(cols)[:64])
    r0, c0 = bad[0]
    diff = (y - ref)[r0, c0].item()
    # is the wrong value some other reference element of the same row?
    hit = (ref[r0] == y[r0, c0]).nonzero().flatten().tolist()
    print(f"  first bad ({r0},{c0}) got {y[r0, c0].item()} want {ref[r0, c0].item()}; equals ref cols {hit[:8]}")

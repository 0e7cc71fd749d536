#!/usr/bin/env python3
"""Debug probe for the four-wave tile: one-hot activations X[t][k] = (k == t mod K) make Y[t][n] = W[n][t mod K], so
with W[n][k] = n the output names the weight ROW that reached (t, n), and with W[n][k] = k / 8 the k granule."""
import os
import sys
from collections import Counter

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from xotorch_support_jetson_amd.ops._ext import require  # noqa: E402
from xotorch_support_jetson_amd.ops.weights_layout import shuffle_for_stream  # noqa: E402

C = require()
M, N, K = 256, 256, int(sys.argv[1]) if len(sys.argv) > 1 else 128
t = torch.arange(M)
X = torch.zeros(M, K)
X[t, t % K] = 1.0
X = X.to(torch.bfloat16).cuda()
for what in ("row", "kgran"):
  if what == "row":
    W = torch.arange(N).float().view(N, 1).expand(N, K).contiguous()
  else:
    W = (torch.arange(K) // 8).float().view(1, K).expand(N, K).contiguous()
  W = W.to(torch.bfloat16).cuda()
  y = torch.zeros(M, N, device="cuda", dtype=torch.float32)
  C.gemm_big(X, shuffle_for_stream(W), y, None, None, None, 0, 4256, 1)
  ref = X.float() @ W.float().t()
  bad = (y != ref).nonzero().tolist()
  print(what, "K", K, "wrong", len(bad))
  c = Counter()
  for r, n in bad[:20000]:
    c[(r % 16, n % 128, int(ref[r, n].item()), int(y[r, n].item()))] += 1
  for k, v in c.most_common(25):
    print("  (row%16, col%128, want, got)", k, v)

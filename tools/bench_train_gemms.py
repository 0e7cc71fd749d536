#!/usr/bin/env python3
"""The training GEMMs of one Llama-3-8B layer micro-batch (T tokens) on the own MFMA kernels (ops/linear.py policy
over gemm_big / stream-K, operands relaid by csrc/layout.hip) vs torch.matmul (hipBLASLt), per role:
  fwd  y = x W^T          dX  dY W          dW  dY^T X (accumulating: beta = 1 / residual epilogue)
  python tools/bench_train_gemms.py [--tokens 2048] [--model llama-3-8b]   -> one JSON line per shape/role"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=20):
  for _ in range(3):
    fn()
  torch.cuda.synchronize()
  a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
  a.record()
  for _ in range(iters):
    fn()
  b.record()
  torch.cuda.synchronize()
  return a.elapsed_time(b) / iters * 1e3  # us


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument("--tokens", type=int, default=2048)
  ap.add_argument("--model", default="llama-3-8b")
  a = ap.parse_args()
  from xotorch_support_jetson_amd.models.config import preset
  from xotorch_support_jetson_amd.ops.linear import linear
  from xotorch_support_jetson_amd.train.autograd_ops import TrainWeight, relayout
  c = preset(a.model)
  D, F, H, Hkv, Dh = c.hidden_size, c.intermediate_size, c.num_heads, c.num_kv_heads, c.head_dim
  shapes = {"qkv": ((H + 2 * Hkv) * Dh, D), "o": (D, H * Dh), "gu": (2 * F, D), "down": (D, F), "head": (c.vocab_size, D)}
  T = a.tokens
  dev = "cuda"
  for name, (N, K) in shapes.items():
    w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
    tw = TrainWeight(w)
    x = torch.randn(T, K, device=dev, dtype=torch.bfloat16)
    dy = torch.randn(T, N, device=dev, dtype=torch.bfloat16)
    acc = torch.zeros(N, K, device=dev, dtype=torch.bfloat16)
    fl = 2.0 * T * N * K
    res = {}
    res["fwd_own"] = timeit(lambda: linear(x, tw.ws))
    res["fwd_blas"] = timeit(lambda: x @ w.t())
    res["dx_own"] = timeit(lambda: linear(dy, tw.wts))
    res["dx_blas"] = timeit(lambda: dy @ w)
    res["relayout_dw"] = timeit(lambda: (relayout(dy, 2), relayout(x, 1)))
    dyt, xts = relayout(dy, 2), relayout(x, 1)
    res["dw_own"] = timeit(lambda: linear(dyt, xts, residual=acc, epi="resid", out=acc))
    res["dw_own_fresh"] = timeit(lambda: linear(dyt, xts, out=acc))
    res["dw_blas"] = timeit(lambda: acc.addmm_(dy.t(), x))
    out = {"shape": name, "N": N, "K": K, "T": T}
    for k, us in res.items():
      out[k + "_us"] = round(us, 1)
      if not k.startswith("relayout"):
        out[k + "_pflops"] = round(fl / us / 1e9, 3)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
  main()

#!/usr/bin/env python3
"""Weight-gradient GEMM dW = dY^T . X of one Llama-3-8B micro-batch (T = 4096 tokens) per projection, in isolation:
the relayout path (dY^T + shuffle(X^T) by csrc/layout.hip, then the pre-shuffled tile the tuner picks) against the
TN tile (csrc/gemm_w4.hip TN: token-major operands, transposed LDS reads).  Medians of --reps calls, us.

  python tools/bench_dw.py [--T 4096] [--reps 20]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, reps):
  ts = []
  for _ in range(reps):
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    fn()
    en.record()
    en.synchronize()
    ts.append(st.elapsed_time(en) * 1e3)
  ts.sort()
  return round(ts[len(ts) // 2], 1)


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument("--T", type=int, default=4096)
  ap.add_argument("--reps", type=int, default=20)
  ap.add_argument("--only", default="", help="one projection (qkv / o / gate_up / down)")
  a = ap.parse_args()
  from xotorch_support_jetson_amd.ops._ext import require
  from xotorch_support_jetson_amd.ops.linear import linear
  from xotorch_support_jetson_amd.train.autograd_ops import relayout
  C = require()
  dev = torch.device("cuda", 0)
  T = a.T
  for name, M, N in (("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 28672, 4096), ("down", 4096, 14336)):
    if a.only and name != a.only:
      continue
    dy = torch.randn(T, M, device=dev).to(torch.bfloat16)
    x = torch.randn(T, N, device=dev).to(torch.bfloat16)
    acc = torch.zeros(M, N, device=dev, dtype=torch.bfloat16)
    dyt, xts = relayout(dy, 2), relayout(x, 1)
    linear(dyt, xts, residual=acc, epi="resid", out=acc)  # tune once
    C.gemm_tn(dy, x, acc, True)
    r = {"op": name, "M": M, "N": N, "T": T}
    r["relayout_us"] = timed(lambda: (relayout(dy, 2, dyt), relayout(x, 1, xts)), a.reps)
    r["gemm_shuffled_us"] = timed(lambda: linear(dyt, xts, residual=acc, epi="resid", out=acc), a.reps)
    r["tn_us"] = timed(lambda: C.gemm_tn(dy, x, acc, True), a.reps)
    fl = 2.0 * M * N * T
    r["tn_TFs"] = round(fl / r["tn_us"] / 1e6, 1)
    r["shuffled_TFs"] = round(fl / r["gemm_shuffled_us"] / 1e6, 1)
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
  main()

#!/usr/bin/env python3
"""Per-tile fixed cost of gemm_big vs its per-k-step cost: one round of 256 tiles (M = N = 4096) at K = 128 ..
8192, plain / residual / fp32-out epilogues, and hipBLASLt at the same shapes.  t(K) = fixed + per_step * K / 64
(least squares); 'fixed' is the prologue + epilogue + launch of one tile per CU.  Random operands, weights
resident (the K sweep stays within the 256 MB cache).

  python tools/lab/gemm_overhead.py [--codes 2256,256] [--m 4096] [--n 4096]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def t_us(fn, iters=30):
  for _ in range(3):
    fn()
  torch.cuda.synchronize()
  st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
  best = float("inf")
  for _ in range(3):
    st.record()
    for _ in range(iters):
      fn()
    en.record()
    en.synchronize()
    best = min(best, st.elapsed_time(en) * 1e3 / iters)
  return best


def fit(ks, ts):
  n = len(ks)
  xs = [k / 64 for k in ks]
  mx, my = sum(xs) / n, sum(ts) / n
  b = sum((x - mx) * (y - my) for x, y in zip(xs, ts)) / sum((x - mx) ** 2 for x in xs)
  return my - b * mx, b


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument("--codes", default="2256,256")
  ap.add_argument("--m", type=int, default=4096)
  ap.add_argument("--n", type=int, default=4096)
  ap.add_argument("--ks", default="128,256,512,1024,2048,4096,8192")
  a = ap.parse_args()
  from xotorch_support_jetson_amd.ops import kernels as K
  from xotorch_support_jetson_amd.ops._ext import require
  from xotorch_support_jetson_amd.ops.weights_layout import shuffle_for_stream
  C = require()
  dev = torch.device("cuda:0")
  M, N = a.m, a.n
  ks = [int(k) for k in a.ks.split(",")]
  for code in [int(c) for c in a.codes.split(",")]:
    for epi, f32 in (("none", False), ("resid", False), ("none", True)):
      ts, tb = [], []
      for Kd in ks:
        x = torch.randn(M, Kd, device=dev, dtype=torch.bfloat16)
        w = torch.randn(N, Kd, device=dev, dtype=torch.bfloat16) * 0.02
        ws_ = shuffle_for_stream(w)
        r = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
        y = torch.empty(M, N, device=dev, dtype=torch.float32 if f32 else torch.bfloat16)
        res = r if epi == "resid" else None
        ts.append(t_us(lambda: C.gemm_big(x, ws_, y, None, res, None, K.EPI[epi], code, 1)))
        if epi == "resid":
          tb.append(t_us(lambda: torch.addmm(r, x, w.t(), out=y)))
        elif f32:
          tb.append(float("nan"))
        else:
          tb.append(t_us(lambda: torch.mm(x, w.t(), out=y)))
      fixed, step = fit(ks, ts)
      out = {"code": code, "epi": epi, "out_f32": f32, "M": M, "N": N, "ks": ks, "own_us": [round(t, 1) for t in ts],
             "blas_us": [round(t, 1) for t in tb], "fixed_us": round(fixed, 2), "per_kstep_us": round(step, 4)}
      if not f32:
        fb, sb = fit(ks, tb)
        out.update(blas_fixed_us=round(fb, 2), blas_per_kstep_us=round(sb, 4))
      print(json.dumps(out), flush=True)


if __name__ == "__main__":
  main()

#!/usr/bin/env python3
"""Training attention kernels in isolation at the Llama-3-8B training shape (B=2, L=2048, 32 / 8 heads of 128):
forward, and the backward (dQ + dK/dV + reduce), median of N timed repetitions on one stream.  (The round-5 v1
backward kernels this used to A/B against were removed in round 6; their numbers are in profiles/r5/train/.)

  python tools/bench_attn_train.py [--B 2 --L 2048 --H 32 --Hkv 8 --Dh 128 --reps 20]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument("--B", type=int, default=2)
  ap.add_argument("--L", type=int, default=2048)
  ap.add_argument("--H", type=int, default=32)
  ap.add_argument("--Hkv", type=int, default=8)
  ap.add_argument("--Dh", type=int, default=128)
  ap.add_argument("--reps", type=int, default=20)
  a = ap.parse_args()
  from xotorch_support_jetson_amd.train import autograd_ops as A
  dev = torch.device("cuda", 0)
  B, L, H, Hkv, Dh = a.B, a.L, a.H, a.Hkv, a.Dh
  torch.manual_seed(0)
  qkv = (torch.randn(B * L, (H + 2 * Hkv) * Dh, device=dev) * 0.5).to(torch.bfloat16).requires_grad_()
  do = torch.randn(B * L, H * Dh, device=dev).to(torch.bfloat16)

  def fwd():
    return A.attention(qkv[:, :H * Dh], qkv[:, H * Dh:(H + Hkv) * Dh], qkv[:, (H + Hkv) * Dh:], B, L, H, Hkv, Dh)

  def timed(fn):
    ts = []
    for i in range(a.reps + 3):
      e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
      e0.record()
      fn()
      e1.record()
      torch.cuda.synchronize()
      if i >= 3:
        ts.append(e0.elapsed_time(e1) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]

  with torch.no_grad():
    t_fwd = timed(fwd)
  o = fwd()

  def bwd():
    qkv.grad = None
    torch.autograd.backward(o, do, retain_graph=True)
  t_bwd = timed(bwd)
  flops = 4 * B * H * Dh * L * L / 2  # causal: two L x L x Dh products, half the square
  print(json.dumps({"shape": [B, L, H, Hkv, Dh], "fwd_us": round(t_fwd, 1), "bwd_us": round(t_bwd, 1),
                    "fwd_tflops": round(flops / t_fwd / 1e6, 1), "bwd_tflops": round(2.5 * flops / t_bwd / 1e6, 1)}))


if __name__ == "__main__":
  main()

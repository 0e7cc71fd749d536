#!/usr/bin/env python3
"""The training step's operand relayouts in isolation (csrc/layout.hip), at the Llama-3-8B shapes of one 4096-token
micro-batch: dY^T (transpose) and shuffle(X^T) (shuffle_t) of every projection, variant 1 (128 x 64 tiles staged
transposed, row-fastest grid) vs variant 2 (128 x 128 tiles read back with ds_read_b64_tr_b16, column-fastest grid).

  python tools/bench_layout.py [--T 4096] [--reps 30]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument("--T", type=int, default=4096)
  ap.add_argument("--reps", type=int, default=30)
  a = ap.parse_args()
  from xotorch_support_jetson_amd.ops._ext import require
  C = require()
  dev = torch.device("cuda", 0)
  out = {}
  for name, cols in (("qkv_dy", 6144), ("o_dy", 4096), ("gu_dy", 28672), ("down_x", 14336)):
    src = torch.randn(a.T, cols, device=dev).to(torch.bfloat16)
    dst = torch.empty(cols, a.T, device=dev, dtype=torch.bfloat16)
    for mode, mname in ((2, "transpose"), (1, "shuffle_t")):
      for variant in (1, 2):
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        C.relayout(src, dst, mode, variant)
        torch.cuda.synchronize()
        st.record()
        for _ in range(a.reps):
          C.relayout(src, dst, mode, variant)
        en.record()
        en.synchronize()
        us = st.elapsed_time(en) * 1e3 / a.reps
        out[f"{name}_{mname}_v{variant}"] = {"us": round(us, 1), "TBps": round(2 * src.numel() * 2 / us / 1e6, 2)}
  print(json.dumps(out), flush=True)


if __name__ == "__main__":
  main()

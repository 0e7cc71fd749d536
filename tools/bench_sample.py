"""On-device sampling at Llama-3 vocab: one workgroup per row vs chunk candidates + merge.

  python tools/bench_sample.py [--json out.json]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from xotorch_support_jetson_amd.ops._ext import require  # noqa: E402


def t_us(fn, iters=20):
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


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument("--json", default=None)
  args = ap.parse_args()
  C = require()
  dev = torch.device("cuda:0")
  V, k = 128256, 35
  rows = []
  for B in (1, 16, 64, 128, 256, 512):
    logits = torch.randn(B, V, device=dev) * 3
    temps = torch.full((B,), 0.6, device=dev)
    so = torch.tensor([1234, 7], dtype=torch.int64, device=dev)
    outs = {}
    r = dict(B=B)
    for algo in (0, 1, 2):
      o = torch.empty(B, dtype=torch.int32, device=dev)
      r[f"us_algo{algo}"] = round(t_us(lambda: C.sample(logits, temps, k, so, o, algo)), 1)
      outs[algo] = o.clone()
    r["same_tokens"] = bool((outs[0] == outs[1]).all().item() and (outs[0] == outs[2]).all().item())
    rows.append(r)
    print(json.dumps(r), flush=True)
  if args.json:
    json.dump(rows, open(args.json, "w"), indent=1)


if __name__ == "__main__":
  main()

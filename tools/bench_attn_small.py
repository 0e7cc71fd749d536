"""Decode attention at small batches (latency regime): workgroup kernel (algo 0) vs wave kernel
(algo 2, and 3 with non-temporal page loads) over partition sizes, each timed as 20 calls replayed from one HIP graph.

  python tools/bench_attn_small.py [--json out.json]
"""
import argparse
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from xotorch_support_jetson_amd.ops import kernels as K  # noqa: E402


def graph_us(fn, reps=20):
  s = torch.cuda.Stream()
  s.wait_stream(torch.cuda.current_stream())
  with torch.cuda.stream(s):
    fn()
  torch.cuda.current_stream().wait_stream(s)
  g = torch.cuda.CUDAGraph()
  with torch.cuda.graph(g):
    for _ in range(reps):
      fn()
  g.replay()
  torch.cuda.synchronize()
  st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
  best = float("inf")
  for _ in range(5):
    st.record()
    g.replay()
    en.record()
    en.synchronize()
    best = min(best, st.elapsed_time(en) * 1e3 / reps)
  return best


def pmc_run(B, ctx, H=64, Hkv=8, Dh=128):
  dev = torch.device("cuda:0")
  pages = -(-ctx // 64)
  npool = B * pages + 4
  kc = torch.randn(npool, Hkv, 64, Dh, device=dev).to(torch.bfloat16)
  vc = torch.randn(npool, Hkv, Dh, 64, device=dev).to(torch.bfloat16)
  bt = torch.randperm(npool, device=dev)[:B * pages].view(B, pages).to(torch.int32).contiguous()
  cl = torch.full((B,), ctx, device=dev, dtype=torch.int32)
  q = torch.randn(B, H, Dh, device=dev).to(torch.bfloat16)
  out = torch.empty_like(q)
  ws = K.DecodeWorkspace(B, H, Dh, pages * 64, dev)
  for _ in range(20):
    K.attn_decode(q, kc, vc, bt, cl, 1 / math.sqrt(Dh), ws, out)
  torch.cuda.synchronize()
  print("cfg", ws.partition(B, Hkv, pages), "KV bytes", 2 * B * Hkv * ctx * Dh * 2)


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument("--json", default=None)
  ap.add_argument("--pmc", default=None, help="B,ctx: only the auto config, 20 direct calls (for rocprofv3 --pmc)")
  args = ap.parse_args()
  if args.pmc:
    B, ctx = (int(v) for v in args.pmc.split(","))
    return pmc_run(B, ctx)
  dev = torch.device("cuda:0")
  H, Hkv, Dh = 64, 8, 128
  rows = []
  for B in (1, 4, 16, 64):
    for ctx in (530, 2048, 8192):
      pages = -(-ctx // 64)
      npool = B * pages + 4
      kc = torch.randn(npool, Hkv, 64, Dh, device=dev).to(torch.bfloat16)
      vc = torch.randn(npool, Hkv, Dh, 64, device=dev).to(torch.bfloat16)
      bt = torch.randperm(npool, device=dev)[:B * pages].view(B, pages).to(torch.int32).contiguous()
      cl = torch.full((B,), ctx, device=dev, dtype=torch.int32)
      q = torch.randn(B, H, Dh, device=dev).to(torch.bfloat16)
      out = torch.empty_like(q)
      r = dict(B=B, ctx=ctx)
      for algo, ppps in ((0, (4, 8, 16, 32)), (2, (2, 4, 8, 16)), (3, (2, 4, 8, 16))):
        for ppp in ppps:
          ws = K.DecodeWorkspace(B, H, Dh, pages * 64, dev, pages_per_part=ppp, algo=algo)
          r[f"a{algo}_p{ppp}_r"] = round(graph_us(lambda: K.attn_decode(q, kc, vc, bt, cl, 1 / math.sqrt(Dh), ws, out)), 2)
      ws = K.DecodeWorkspace(B, H, Dh, pages * 64, dev)
      r["auto"] = round(graph_us(lambda: K.attn_decode(q, kc, vc, bt, cl, 1 / math.sqrt(Dh), ws, out)), 2)
      r["auto_cfg"] = list(ws.partition(B, Hkv, pages))
      rows.append(r)
      print(json.dumps(r), flush=True)
  if args.json:
    json.dump(rows, open(args.json, "w"), indent=1)


if __name__ == "__main__":
  main()

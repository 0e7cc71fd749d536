"""Does the KV page layout limit decode attention at the headline?  The pool stores a page as [Hkv][64][Dh], so the
pages one (sequence, KV head) unit walks are 16 KB pieces Hkv x 16 KB apart.  Same bytes, same unit count, four
placements: Llama-3-70B heads (8 KV heads) with random / per-sequence contiguous block tables, and the same work
as 8x the sequences of ONE KV head each (a unit's pages then contiguous 16 KB after 16 KB -- what a head-major
pool [Hkv][pages] would give), random / contiguous.  Each timed as 20 calls replayed from one HIP graph.

  python tools/bench_attn_layout.py [--json out.json]
"""
import argparse
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from xotorch_support_jetson_amd.ops import kernels as K  # noqa: E402
from tools.bench_attn_small import graph_us  # noqa: E402


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument("--json", default=None)
  args = ap.parse_args()
  dev = torch.device("cuda:0")
  Dh, G, ctx = 128, 8, 531
  pages = -(-ctx // 64)
  rows = []
  for B, Hkv in ((512, 8), (4096, 1)):
    H = G * Hkv
    npool = B * pages + 4
    kc = torch.randn(npool, Hkv, 64, Dh, device=dev).to(torch.bfloat16)
    vc = torch.randn(npool, Hkv, Dh, 64, device=dev).to(torch.bfloat16)
    q = torch.randn(B, H, Dh, device=dev).to(torch.bfloat16)
    out = torch.empty_like(q)
    cl = torch.full((B,), ctx, device=dev, dtype=torch.int32)
    kv_bytes = 2 * B * Hkv * ctx * Dh * 2
    ws = K.DecodeWorkspace(B, H, Dh, pages * 64, dev)
    for place in ("random", "contiguous"):
      if place == "random":
        bt = torch.randperm(npool, device=dev)[:B * pages]
      else:
        bt = torch.arange(B * pages, device=dev)
      bt = bt.view(B, pages).to(torch.int32).contiguous()
      us = graph_us(lambda: K.attn_decode(q, kc, vc, bt, cl, 1 / math.sqrt(Dh), ws, out))
      r = dict(B=B, Hkv=Hkv, H=H, pages=place, us=round(us, 1), tbps=round(kv_bytes / us / 1e6, 2),
               part=list(ws.partition(B, Hkv, pages)))
      print(json.dumps(r), flush=True)
      rows.append(r)
    del kc, vc
    torch.cuda.empty_cache()
  if args.json:
    with open(args.json, "w") as f:
      json.dump(rows, f, indent=1)


if __name__ == "__main__":
  main()

"""Decode attention at the headline batch (B = 512 sequences, Llama-3-70B heads, ctx ~ 531): wave kernel
over split-KV partition sizes (pages per partition), each timed as 20 calls replayed from one HIP graph.

  python tools/bench_attn_b512.py [--json out.json]
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
  ap.add_argument("--algos", default="2", help="wave-kernel variants to time (csrc/attention.hip: 1 no prefetch, "
                  "2 / 3 double register set, 5 / 6 one set refilled per half; 3 / 6 nt loads)")
  args = ap.parse_args()
  dev = torch.device("cuda:0")
  H, Hkv, Dh = 64, 8, 128
  rows = []
  for B, ctx in ((512, 531), (256, 1040), (128, 2048)):
    pages = -(-ctx // 64)
    npool = B * pages + 4
    kc = torch.randn(npool, Hkv, 64, Dh, device=dev).to(torch.bfloat16)
    vc = torch.randn(npool, Hkv, Dh, 64, device=dev).to(torch.bfloat16)
    bt = torch.randperm(npool, device=dev)[:B * pages].view(B, pages).to(torch.int32).contiguous()
    cl = torch.full((B,), ctx, device=dev, dtype=torch.int32)
    q = torch.randn(B, H, Dh, device=dev).to(torch.bfloat16)
    out = torch.empty_like(q)
    kv_bytes = 2 * B * Hkv * ctx * Dh * 2
    auto = K.DecodeWorkspace(B, H, Dh, pages * 64, dev)
    cands = [("auto", auto)]
    for a in [int(x) for x in args.algos.split(",")]:
      cands += [(f"a{a}-ppp{p}", K.DecodeWorkspace(B, H, Dh, pages * 64, dev, pages_per_part=p, algo=a))
                for p in sorted({pages, -(-pages // 2), -(-pages // 3), 2})]
    ref = None
    for name, ws in cands:
      us = graph_us(lambda: K.attn_decode(q, kc, vc, bt, cl, 1 / math.sqrt(Dh), ws, out))
      if ref is None:
        ref = out.float().clone()
      err = ((out.float() - ref).abs().max() / ref.abs().max()).item()
      r = dict(B=B, ctx=ctx, cfg=name, part=list(ws.partition(B, Hkv, pages)), us=round(us, 1),
               tbps=round(kv_bytes / us / 1e6, 2), err_vs_auto=round(err, 5))
      rows.append(r)
      print(json.dumps(r), flush=True)
    del kc, vc
    torch.cuda.empty_cache()
  if args.json:
    with open(args.json, "w") as f:
      json.dump(rows, f, indent=1)


if __name__ == "__main__":
  main()

#!/usr/bin/env python3
"""MLA decode attention micro-benchmark (DeepSeek-V3 shapes: 128 heads, kv_lora 512, rope 64):
  python tools/bench_mla.py --batch 256 --ctx 525 [--heads 128] [--iters 50]
Prints one JSON line per kernel variant (narrow / wide) with µs per call and the latent-cache bytes/s."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument("--batch", type=int, default=256)
  ap.add_argument("--ctx", type=int, default=525)
  ap.add_argument("--heads", type=int, default=128)
  ap.add_argument("--dl", type=int, default=512)
  ap.add_argument("--iters", type=int, default=50)
  ap.add_argument("--variants", default="0,1")
  a = ap.parse_args()
  from xotorch_support_jetson_amd.ops import kernels as K
  dev = torch.device("cuda", 0)
  B, H, DL, DR = a.batch, a.heads, a.dl, 64
  width = -(-a.ctx // 64)
  cache = torch.randn(B * width + 1, 64, DL + DR, device=dev, dtype=torch.bfloat16)
  bt = torch.randperm(B * width, device=dev).int().view(B, width)
  ctx = torch.full((B,), a.ctx, dtype=torch.int32, device=dev)
  cu = torch.arange(B + 1, dtype=torch.int32, device=dev)
  q_lat = torch.randn(H, B, DL, device=dev, dtype=torch.bfloat16)
  q_pe = torch.randn(B, H * DR, device=dev, dtype=torch.bfloat16)
  ws = K.MLAWorkspace(B, H, DL, width * 64, dev)
  out = torch.empty_like(q_lat)
  ref = None
  for v in a.variants.split(","):
    os.environ["XOT_MLA_WIDE"] = v
    for _ in range(3):
      K.mla_attn(q_lat, q_pe, cache, bt, cu, ctx, 0.1, ws, out)
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(a.iters):
      K.mla_attn(q_lat, q_pe, cache, bt, cu, ctx, 0.1, ws, out)
    en.record()
    en.synchronize()
    us = st.elapsed_time(en) * 1e3 / a.iters
    if ref is None:
      ref = out.float().clone()
    err = ((out.float() - ref).norm() / ref.norm()).item()
    byts = B * a.ctx * (DL + DR) * 2
    flops = 2 * B * H * a.ctx * (DL + DR + DL)
    print(json.dumps({"kernel": "wide" if v == "1" else "narrow", "batch": B, "heads": H, "ctx": a.ctx, "us": round(us, 1),
                      "cache_TBps": round(byts / us / 1e6, 2), "TFLOPs": round(flops / us / 1e6, 1),
                      "partition": ws.partition(B, width), "rel_diff_vs_first": round(err, 5)}), flush=True)


if __name__ == "__main__":
  main()

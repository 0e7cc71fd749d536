#!/usr/bin/env python3
"""Causal prefill attention from the paged KV cache vs torch SDPA (same shapes, contiguous K/V):
  python tools/bench_attn_prefill.py --seqs 4 --len 2048 --heads 64 --kv-heads 8 --dh 128
One JSON line per kernel variant: µs per call and TFLOP/s (causal FLOPs: 2 L^2 H Dh per sequence)."""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters):
  for _ in range(3):
    fn()
  torch.cuda.synchronize()
  st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
  st.record()
  for _ in range(iters):
    fn()
  en.record()
  en.synchronize()
  return st.elapsed_time(en) * 1e3 / iters


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument("--seqs", type=int, default=4)
  ap.add_argument("--len", type=int, default=2048)
  ap.add_argument("--heads", type=int, default=64)
  ap.add_argument("--kv-heads", type=int, default=8)
  ap.add_argument("--dh", type=int, default=128)
  ap.add_argument("--iters", type=int, default=20)
  a = ap.parse_args()
  from xotorch_support_jetson_amd.ops import kernels as K
  from xotorch_support_jetson_amd.ops import reference as R
  dev = torch.device("cuda", 0)
  B, L, H, Hkv, Dh = a.seqs, a.len, a.heads, a.kv_heads, a.dh
  pages = -(-L // 64)
  kc = torch.randn(B * pages, Hkv, 64, Dh, device=dev, dtype=torch.bfloat16)
  vc = torch.randn(B * pages, Hkv, Dh, 64, device=dev, dtype=torch.bfloat16)
  bt = torch.randperm(B * pages, device=dev).int().view(B, pages)
  cu = torch.arange(B + 1, device=dev, dtype=torch.int32) * L
  cl = torch.full((B,), L, device=dev, dtype=torch.int32)
  q = torch.randn(B * L, H, Dh, device=dev, dtype=torch.bfloat16)
  scale = Dh ** -0.5
  flops = 2 * B * L * L * H * Dh  # causal: half of 4 L^2 H Dh
  outs = {}
  for algo in (1, 2):
    K.PREFILL_ALGO = algo
    out = torch.empty_like(q)
    us = timeit(lambda: K.attn_prefill(q, kc, vc, bt, cu, cl, L, scale, out=out), a.iters)
    outs[algo] = out.float()
    print(json.dumps({"kernel": f"prefill_v{algo}", "seqs": B, "len": L, "heads": H, "kv_heads": Hkv, "dh": Dh,
                      "us": round(us, 1), "TFLOPs": round(flops / us / 1e6, 1)}), flush=True)
  # torch SDPA on the same data laid out contiguously
  kk = kc[bt.long()].permute(0, 2, 1, 3, 4).reshape(B, Hkv, pages * 64, Dh)[:, :, :L]
  from xotorch_support_jetson_amd.ops.reference import v_chunks
  vv = v_chunks(vc)[bt.long()].permute(0, 2, 1, 3, 5, 4).reshape(B, Hkv, pages * 64, Dh)[:, :, :L]
  kk = kk.repeat_interleave(H // Hkv, 1).contiguous()
  vv = vv.repeat_interleave(H // Hkv, 1).contiguous()
  qq = q.view(B, L, H, Dh).transpose(1, 2).contiguous()
  us = timeit(lambda: F.scaled_dot_product_attention(qq, kk, vv, is_causal=True, scale=scale), a.iters)
  ref = F.scaled_dot_product_attention(qq, kk, vv, is_causal=True, scale=scale).transpose(1, 2).reshape(B * L, H, Dh)
  errs = {k: round(((v - ref.float()).norm() / ref.float().norm()).item(), 5) for k, v in outs.items()}
  print(json.dumps({"kernel": "torch_sdpa", "us": round(us, 1), "TFLOPs": round(flops / us / 1e6, 1),
                    "rel_err_vs_sdpa": errs}), flush=True)


if __name__ == "__main__":
  main()

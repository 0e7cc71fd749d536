#!/usr/bin/env python3
"""The split-K slab consumers of the headline decode step in isolation (Llama-3-70B, 512 sequences): the fused
slab reduce + RoPE + paged KV write after the qkv GEMM (S = 3) and the fused slab reduce + residual + RMSNorm after
the o / down GEMMs (S = 4), with ablations that tell what each costs, against a plain fp32 read of the same slabs.

  python tools/bench_reduce.py [--reps 50]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, reps, flush=None):
  st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
  ts = []
  for _ in range(reps):
    if flush is not None:
      flush()
    st.record()
    fn()
    en.record()
    en.synchronize()
    ts.append(st.elapsed_time(en) * 1e3)
  ts.sort()
  return round(ts[len(ts) // 2], 2)


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument("--reps", type=int, default=50)
  ap.add_argument("--batch", type=int, default=512)
  a = ap.parse_args()
  from xotorch_support_jetson_amd.ops._ext import require
  from xotorch_support_jetson_amd.ops.rope import build_cos_sin
  C = require()
  dev = torch.device("cuda", 0)
  T, H, Hkv, Dh, D = a.batch, 64, 8, 128, 8192
  N = (H + 2 * Hkv) * Dh
  pages = T * 9 + 16
  g = torch.Generator(device=dev).manual_seed(0)
  cs = build_cos_sin(Dh, 4096, 500000.0, None, device=dev)
  kc = torch.zeros(pages, Hkv, 64, Dh, device=dev, dtype=torch.bfloat16)
  vc = torch.zeros(pages, Hkv, Dh, 64, device=dev, dtype=torch.bfloat16)
  pos = torch.full((T,), 530, device=dev, dtype=torch.int32)
  # each sequence's token in its own page (as in the step: ctx 530 -> page 8 of 9, offset 18)
  slots = (torch.randperm(pages - 16, device=dev, generator=g)[:T].to(torch.int64) * 64 + 18)
  no_slots = torch.full_like(slots, -1)
  q = torch.empty(T, H, Dh, device=dev, dtype=torch.bfloat16)
  out = {}
  for S in (3, 4):
    ws = torch.randn(S, T, N, device=dev, generator=g)
    touch = lambda: ws.add_(0.0)  # noqa: E731  (the slabs freshly written, as by the GEMM before the reduce)
    out[f"rope_kv_S{S}_us"] = timed(lambda: C.splitk_rope_kv_write(ws, S, None, pos, cs, slots, q, kc, vc, H, Hkv),
                                    a.reps, touch)
    out[f"rope_q_only_S{S}_us"] = timed(
      lambda: C.splitk_rope_kv_write(ws, S, None, pos, cs, no_slots, q, kc, vc, H, Hkv), a.reps, touch)
    out[f"read_slabs_S{S}_us"] = timed(lambda: ws.sum(0), a.reps, touch)
    out[f"slab_MB_S{S}"] = round(ws.numel() * 4 / 1e6, 1)
  for S in (2, 4):
    ws = torch.randn(S, T, D, device=dev, generator=g)
    h = torch.randn(T, D, device=dev, generator=g).to(torch.bfloat16)
    w = torch.randn(D, device=dev, generator=g).to(torch.bfloat16)
    o = torch.empty_like(h)
    touch = lambda: ws.add_(0.0)  # noqa: E731
    out[f"resid_rmsnorm_S{S}_us"] = timed(lambda: C.splitk_resid_rmsnorm(ws, S, None, h, w, o, 1e-5), a.reps, touch)
    out[f"read_slabs_D_S{S}_us"] = timed(lambda: ws.sum(0), a.reps, touch)
  big = torch.empty(256 << 20, device=dev)
  out["copy_1GB_TBps"] = round(2 * big.numel() * 4 / timed(lambda: big.clone(), 10) / 1e6, 2)
  print(json.dumps(out), flush=True)


if __name__ == "__main__":
  main()

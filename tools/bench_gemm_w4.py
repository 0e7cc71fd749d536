#!/usr/bin/env python3
"""Tall-M GEMMs (prefill chunks, training micro-batches): the four-wave tile (code 4256, csrc/gemm_w4.hip) vs the
two-phase ping-pong 256 x 256 tile (2256) vs hipBLASLt on row-major weights, random operands, weights rotated
through >= 1 GB (HBM-cold, as in a forward pass).  One JSON line per shape:

  python tools/bench_gemm_w4.py [--shapes train8b,prefill70b,decode70b] [--codes 4256,2256]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = {  # name: (M, N, K, epilogue)
  "train8b": [(4096, 6144, 4096, "none"), (4096, 4096, 4096, "resid"), (4096, 28672, 4096, "none"),
              (4096, 4096, 14336, "resid"), (4096, 4096, 28672, "none"), (4096, 14336, 4096, "none"),
              (4096, 128256, 4096, "none")],
  "prefill70b": [(8192, 10240, 8192, "none"), (8192, 8192, 8192, "resid"), (8192, 57344, 8192, "silu"),
                 (8192, 8192, 28672, "resid")],
  "decode70b": [(512, 57344, 8192, "silu"), (512, 8192, 28672, "resid"), (512, 10240, 8192, "none")],
}


def t_us(fn, n, iters=10):
  for i in range(2):
    fn(i % n)
  torch.cuda.synchronize()
  st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
  best = float("inf")
  for _ in range(3):
    st.record()
    for i in range(iters):
      fn(i % n)
    en.record()
    en.synchronize()
    best = min(best, st.elapsed_time(en) * 1e3 / iters)
  return best


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument("--shapes", default="train8b,prefill70b")
  ap.add_argument("--codes", default="4256,2256")
  ap.add_argument("--splits", type=int, default=1)
  ap.add_argument("--mnk", default="", help="one shape M,N,K,epi instead of --shapes (e.g. for PMC passes)")
  ap.add_argument("--no-blas", action="store_true")
  a = ap.parse_args()
  if a.mnk:
    m_, n_, k_, e_ = a.mnk.split(",")
    SHAPES["mnk"] = [(int(m_), int(n_), int(k_), e_)]
    a.shapes = "mnk"
  from xotorch_support_jetson_amd.ops import kernels as K
  from xotorch_support_jetson_amd.ops._ext import require
  from xotorch_support_jetson_amd.ops.weights_layout import shuffle_for_stream
  C = require()
  dev = torch.device("cuda:0")
  torch.manual_seed(0)
  for group in a.shapes.split(","):
    for M, N, Kd, epi in SHAPES[group]:
      nc = max(2, -(-(1 << 30) // (N * Kd * 2)))
      ws_ = [torch.randn(N, Kd, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(nc)]
      wsh = [shuffle_for_stream(w) for w in ws_]
      x = torch.randn(M, Kd, device=dev, dtype=torch.bfloat16)
      r = torch.randn(M, N, device=dev, dtype=torch.bfloat16) if epi == "resid" else None
      y = torch.empty(M, N // 2 if epi == "silu" else N, device=dev, dtype=torch.bfloat16)
      S = a.splits
      slab = torch.empty(S * M * N, device=dev, dtype=torch.float32) if S > 1 else None
      fl = 2.0 * M * N * Kd
      out = {"group": group, "M": M, "N": N, "K": Kd, "epi": epi, "splits": S}
      for code in [int(c) for c in a.codes.split(",") if c != "none"]:
        try:
          us = t_us(lambda i: C.gemm_big(x, wsh[i], y, None, r, slab, K.EPI[epi], code, S), nc)
          out[f"c{code}_us"] = round(us, 1)
          out[f"c{code}_pflops"] = round(fl / us / 1e9, 3)
        except RuntimeError as e:
          out[f"c{code}_err"] = str(e)[:80]
      if a.no_blas:
        print(json.dumps(out), flush=True)
        continue
      if epi == "resid":
        blas = lambda i: torch.addmm(r, x, ws_[i].t())
      else:
        blas = lambda i: x @ ws_[i].t()
      us = t_us(blas, nc)
      out["blas_us"] = round(us, 1)
      out["blas_pflops"] = round(fl / us / 1e9, 3)
      print(json.dumps(out), flush=True)
      del ws_, wsh


if __name__ == "__main__":
  main()

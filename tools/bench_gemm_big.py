"""Large-M GEMM (gemm_big: 256 x BN x 64 LDS-DMA tiles on the pre-shuffled layout) vs the stream GEMM
and hipBLASLt on Llama-3-70B projection shapes, weights rotated through >= 1 GB (HBM-cold, as in a
forward pass).

  python tools/bench_gemm_big.py [--ms 256,512,2048] [--json out.json]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from xotorch_support_jetson_amd.ops import kernels as K  # noqa: E402
from xotorch_support_jetson_amd.ops import linear as L  # noqa: E402
from xotorch_support_jetson_amd.ops._ext import require  # noqa: E402
from xotorch_support_jetson_amd.ops.weights_layout import shuffle_for_stream  # noqa: E402

SHAPES = {"qkv": (10240, 8192, "none"), "o": (8192, 8192, "resid"), "gate_up": (57344, 8192, "silu"),
          "down": (8192, 28672, "resid")}


def t_us(fn, n_copies, iters=20):
  for i in range(3):
    fn(i % n_copies)
  torch.cuda.synchronize()
  st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
  best = float("inf")
  for _ in range(3):
    st.record()
    for i in range(iters):
      fn(i % n_copies)
    en.record()
    en.synchronize()
    best = min(best, st.elapsed_time(en) * 1e3 / iters)
  return best


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument("--ms", default="256,512,2048")
  ap.add_argument("--ops", default=",".join(SHAPES))
  ap.add_argument("--json", default=None)
  args = ap.parse_args()
  dev = torch.device("cuda:0")
  torch.manual_seed(0)
  C = require()
  rows = []
  ws_buf = torch.empty(8 * 4096 * 57344 // 4, dtype=torch.float32, device=dev)
  for name in args.ops.split(","):
    N, Kd, epi = SHAPES[name]
    nc = max(2, -(-(1 << 30) // (N * Kd * 2)))
    wl = [(torch.randn(N, Kd, device=dev) * 0.02).to(torch.bfloat16) for _ in range(nc)]
    wsl = []
    for w in wl:
      s = shuffle_for_stream(w)
      s.xot_layout = "stream"
      wsl.append(s)
    for M in [int(m) for m in args.ms.split(",")]:
      x = torch.randn(M, Kd, device=dev).to(torch.bfloat16)
      res = torch.randn(M, N, device=dev).to(torch.bfloat16) if epi == "resid" else None
      ncol = N // 2 if epi == "silu" else N
      out = torch.empty(M, ncol, dtype=torch.bfloat16, device=dev)
      ref = L._blas(x, wl[0], None, res, epi, None, torch.bfloat16).float()
      flop = 2 * M * N * Kd
      big = {}
      for bn in (256, 1256, 128):
        if N % (bn % 1000):
          continue
        tiles = -(-M // 256) * (N // (bn % 1000))
        for S in (1, 2, 3, 4, 6, 8):
          if S > 1 and (tiles * S > 1024 or S * M * N > ws_buf.numel()):
            continue
          if S > 1 and tiles >= 512:
            continue
          fn = lambda i: C.gemm_big(x, wsl[i], out, None, res, ws_buf if S > 1 else None, K.EPI[epi], bn, S)
          fn(0)
          err = ((out.float() - ref).abs().max() / ref.abs().max()).item()
          us = t_us(fn, nc)
          big[(bn, S)] = (us, err)
      best = min(big, key=lambda k: big[k][0])
      us_big, err_big = big[best]
      us_blas = t_us(lambda i: L._blas(x, wl[i], None, res, epi, None, torch.bfloat16), nc)
      row = dict(op=name, M=M, N=N, K=Kd, big_cfg=list(best), us_big=round(us_big, 1), us_hipblaslt=round(us_blas, 1),
                 tflops_big=round(flop / us_big / 1e6, 1), tflops_blas=round(flop / us_blas / 1e6, 1),
                 rel_err_big=err_big, all_big={f"{k[0]}x{k[1]}": round(v[0], 1) for k, v in big.items()})
      cfg = L.policy.shuffled_cfg(x, wsl[0], None, res, epi, torch.bfloat16)  # what linear() runs
      us_pol = t_us(lambda i: L._shuffled_call(x, wsl[i], None, res, epi, out, cfg), nc)
      L._shuffled_call(x, wsl[0], None, res, epi, out, cfg)
      err = ((out.float() - ref).abs().max() / ref.abs().max()).item()
      row.update(policy_cfg=list(cfg), us_policy=round(us_pol, 1), tflops_policy=round(flop / us_pol / 1e6, 1),
                 rel_err_policy=err)
      rows.append(row)
      print(json.dumps(row), flush=True)
  if args.json:
    with open(args.json, "w") as f:
      json.dump(rows, f, indent=1)


if __name__ == "__main__":
  main()

"""Stream GEMM (pre-shuffled weights, autotuned ntw/split-K, M-blocked) vs hipBLASLt on Llama-3-70B
projection shapes across M (decode batch sizes and small prefill chunks).

  python tools/bench_gemm_m.py [--ms 128,256,512] [--json out.json]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from xotorch_support_jetson_amd.ops import linear as L  # noqa: E402
from xotorch_support_jetson_amd.ops.weights_layout import shuffle_for_stream, unshuffle_from_stream  # noqa: E402

SHAPES = {"qkv": (10240, 8192, "none"), "o": (8192, 8192, "resid"), "gate_up": (57344, 8192, "silu"),
          "down": (8192, 28672, "resid")}


def t_us(fn, n_copies, iters=24):
  """fn(i) uses weight copy i; rotating through >= 1 GB of weights keeps them out of the 256 MB MALL,
  as in a real forward pass (80 layers x 1.7 GB)."""
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
  ap.add_argument("--ms", default="64,128,192,256,384,512")
  ap.add_argument("--json", default=None)
  args = ap.parse_args()
  dev = torch.device("cuda:0")
  torch.manual_seed(0)
  rows = []
  for name, (N, K, epi) in SHAPES.items():
    nc = max(2, -(-(1 << 30) // (N * K * 2)))
    wl = [(torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16) for _ in range(nc)]
    wsl = []
    for w in wl:
      ws = shuffle_for_stream(w)
      ws.xot_layout = "stream"
      wsl.append(ws)
    w, ws = wl[0], wsl[0]
    for M in [int(m) for m in args.ms.split(",")]:
      x = (torch.randn(M, K, device=dev)).to(torch.bfloat16)
      res = torch.randn(M, N, device=dev).to(torch.bfloat16) if epi == "resid" else None
      ncol = N // 2 if epi == "silu" else N
      out = torch.empty(M, ncol, dtype=torch.bfloat16, device=dev)
      L.STREAM_MAX_M = 1 << 30
      cfg = L.policy.shuffled_cfg(x, ws, None, res, epi, torch.bfloat16)
      us_stream = t_us(lambda i: L._shuffled_call(x, wsl[i], None, res, epi, out, cfg), nc)
      # correctness vs hipBLASLt on the row-major weight
      ref = L._blas(x, w, None, res, epi, None, torch.bfloat16)
      L._shuffled_call(x, ws, None, res, epi, out, cfg)
      err = ((out.float() - ref.float()).abs().max() / ref.float().abs().max()).item()
      us_blas = t_us(lambda i: L._blas(x, wl[i], None, res, epi, None, torch.bfloat16), nc)
      us_unshuf = t_us(lambda i: unshuffle_from_stream(wsl[i]), nc)
      gb = (N * K * 2) / 1e9
      row = dict(op=name, M=M, N=N, K=K, cfg=list(cfg), us_stream=round(us_stream, 1), us_hipblaslt=round(us_blas, 1),
                 us_unshuffle_copy=round(us_unshuf, 1), tbps_stream=round(gb / us_stream * 1e3, 2), tbps_blas=round(gb / us_blas * 1e3, 2),
                 tflops_stream=round(2 * M * N * K / us_stream / 1e6, 1), speedup=round(us_blas / us_stream, 2),
                 rel_err=err)
      rows.append(row)
      print(json.dumps(row), flush=True)
  if args.json:
    with open(args.json, "w") as f:
      json.dump(rows, f, indent=1)


if __name__ == "__main__":
  main()

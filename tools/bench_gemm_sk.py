"""Stream-K GEMM (csrc/gemm_sk.hip) vs gemm_big's best configuration vs hipBLASLt on the projection shapes of
Llama-3-70B / 8B, weights rotated through >= 1 GB (HBM-cold, as in a forward pass), random operands.
Checks each output against an fp32 torch reference and the stream-K output for run-to-run determinism.

  python tools/bench_gemm_sk.py [--ms 512,2048] [--ops gate_up,down] [--json out.json]
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
          "down": (8192, 28672, "resid"), "gate_up_8b": (28672, 4096, "silu"), "qkv_8b": (6144, 4096, "none"),
          "down_8b": (4096, 14336, "resid")}


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
  ap.add_argument("--ms", default="512,2048")
  ap.add_argument("--ops", default="gate_up,down,qkv,o")
  ap.add_argument("--json", default=None)
  ap.add_argument("--no-big", action="store_true")
  args = ap.parse_args()
  dev = torch.device("cuda:0")
  torch.manual_seed(0)
  C = require()
  part = torch.empty(C.gemm_sk_part_elems(), dtype=torch.float32, device=dev)
  sync = torch.zeros(1 << 16, dtype=torch.int32, device=dev)
  ws_buf = torch.empty(8 * 4096 * 57344 // 4, dtype=torch.float32, device=dev)
  rows = []
  for name in args.ops.split(","):
    N, Kd, epi = SHAPES[name]
    nc = max(2, -(-(1 << 30) // (N * Kd * 2)))
    wl = [(torch.randn(N, Kd, device=dev) * 0.02).to(torch.bfloat16) for _ in range(nc)]
    wsl = [shuffle_for_stream(w) for w in wl]
    for M in [int(m) for m in args.ms.split(",")]:
      x = torch.randn(M, Kd, device=dev).to(torch.bfloat16)
      res = torch.randn(M, N, device=dev).to(torch.bfloat16) if epi == "resid" else None
      ncol = N // 2 if epi == "silu" else N
      out = torch.empty(M, ncol, dtype=torch.bfloat16, device=dev)
      ref = x.float() @ wl[0].float().t()
      if epi == "silu":  # gate / up interleaved in 16-row groups
        r4 = ref.view(M, N // 32, 2, 16)
        ref = (torch.nn.functional.silu(r4[:, :, 0]) * r4[:, :, 1]).reshape(M, N // 2)
      elif epi == "resid":
        ref = ref + res.float()
      flop = 2 * M * N * Kd
      row = dict(op=name, M=M, N=N, K=Kd)
      # stream-K
      fn = lambda i: C.gemm_sk(x, wsl[i], out, None, res, part, sync, K.EPI[epi], 256)
      fn(0)
      torch.cuda.synchronize()
      err = ((out.float() - ref).abs().max() / ref.abs().max()).item()
      first = out.clone()
      for _ in range(3):
        fn(0)
      det = bool(torch.equal(first, out))
      us = t_us(fn, nc)
      row.update(us_sk=round(us, 1), tflops_sk=round(flop / us / 1e6, 1), rel_err_sk=err, deterministic_sk=det,
                 sync_clean=bool((sync == 0).all().item()))
      # gemm_big best
      if not args.no_big:
        big = {}
        for bn in (256, 1256, 128):
          if N % (bn % 1000):
            continue
          tiles = -(-M // 256) * (N // (bn % 1000))
          for S in (1, 2, 3, 4, 6, 8):
            if S > 1 and (tiles * S > 1024 or S * M * N > ws_buf.numel() or tiles >= 512):
              continue
            f2 = lambda i: C.gemm_big(x, wsl[i], out, None, res, ws_buf if S > 1 else None, K.EPI[epi], bn, S)
            f2(0)
            big[(bn, S)] = t_us(f2, nc)
        row.update(big_all={f"{b}x{s}": round(v, 1) for (b, s), v in big.items()})
        best = min(big, key=big.get)
        row.update(big_cfg=list(best), us_big=round(big[best], 1), tflops_big=round(flop / big[best] / 1e6, 1))
      ub = t_us(lambda i: L._blas(x, wl[i], None, res, epi, None, torch.bfloat16), nc)
      row.update(us_hipblaslt=round(ub, 1), tflops_blas=round(flop / ub / 1e6, 1))
      rows.append(row)
      print(json.dumps(row), flush=True)
    del wl, wsl
    torch.cuda.empty_cache()
  if args.json:
    with open(args.json, "w") as f:
      json.dump(rows, f, indent=1)


if __name__ == "__main__":
  main()

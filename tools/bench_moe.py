"""Grouped expert GEMMs (Mixtral-8x7B shapes) in isolation: weight-streaming kernel vs gemm_big tiles,
against the same work as per-expert dense GEMMs.

  python tools/bench_moe.py [--tokens 512] [--json out.json]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from xotorch_support_jetson_amd.ops import linear as L  # noqa: E402
from xotorch_support_jetson_amd.ops._ext import require  # noqa: E402
from xotorch_support_jetson_amd.ops.weights_layout import shuffle_for_stream  # noqa: E402


def t_us(fn, iters=10):
  fn()
  torch.cuda.synchronize()
  st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
  best = float("inf")
  for _ in range(3):
    st.record()
    for _ in range(iters):
      fn()
    en.record()
    en.synchronize()
    best = min(best, st.elapsed_time(en) * 1e3 / iters)
  return best


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument("--tokens", default="1,64,512")
  ap.add_argument("--json", default=None)
  args = ap.parse_args()
  dev = torch.device("cuda:0")
  C = require()
  E, k, D, F = 8, 2, 4096, 14336
  # weights rotated over 2 layer copies (3.8 GB each) so they stream from HBM
  gus = [torch.stack([shuffle_for_stream((torch.randn(2 * F, D, device=dev) * 0.02).to(torch.bfloat16))
                      for _ in range(E)]) for _ in range(2)]
  dws = [torch.stack([shuffle_for_stream((torch.randn(D, F, device=dev) * 0.02).to(torch.bfloat16))
                      for _ in range(E)]) for _ in range(2)]
  rows = []
  for T in [int(t) for t in args.tokens.split(",")]:
    x = torch.randn(T, D, device=dev).to(torch.bfloat16)
    logits = torch.randn(T, E, device=dev)
    topw = torch.empty(T * k, device=dev)
    topi = torch.empty(T * k, dtype=torch.int32, device=dev)
    slot_of = torch.empty_like(topi)
    sorted_tok = torch.empty_like(topi)
    off = torch.empty(E + 1, dtype=torch.int32, device=dev)
    C.moe_route(logits, k, topw, topi, slot_of, sorted_tok, off)
    act = torch.empty(T * k, F, dtype=torch.bfloat16, device=dev)
    hist = (off[1:] - off[:-1]).tolist()
    gb_gu, gb_dn = E * 2 * F * D * 2 / 1e9, E * D * F * 2 / 1e9
    r = dict(T=T, rows_per_expert=hist)
    it = [0]

    def nxt():
      it[0] ^= 1
      return it[0]

    for bm in (0, 128, 192, 256, 1128, 1192, 1256):  # + 1000: deeper LDS pipeline (more weight bytes in flight)
      if bm and T * k < 16:
        continue
      C.gemm_moe(x, gus[0], act, off, sorted_tok, 2, T, True, 1, bm)
      if bm == 0:
        ref = act.float().clone()
      else:  # every tile variant reproduces the weight-streaming kernel's rows
        r[f"gu_relerr_bm{bm}"] = float((act.float() - ref).norm() / ref.norm())
      us = t_us(lambda: C.gemm_moe(x, gus[nxt()], act, off, sorted_tok, 2, T, True, 1, bm))
      r[f"gu_us_bm{bm}"] = round(us, 1)
      r[f"gu_tbps_bm{bm}"] = round(gb_gu / us * 1e3, 2)
      for S in (1, 2, 4, 6, 8):
        y = torch.empty(S * T * k, D, dtype=torch.float32, device=dev)
        try:
          us = t_us(lambda: C.gemm_moe(act, dws[nxt()], y, off, None, 0, T, True, S, bm))
        except RuntimeError:  # split count not supported by this kernel / shape
          continue
        r[f"dn_us_bm{bm}_S{S}"] = round(us, 1)
    # the same bytes as one dense GEMM at M = T*k/E rows per expert, E times
    m = max(1, T * k // E)
    xd = torch.randn(m, D, device=dev).to(torch.bfloat16)
    w0 = gus[0][0]
    w0.xot_layout = "stream"
    cfg = L.policy.shuffled_cfg(xd, w0, None, None, "silu", torch.bfloat16)
    yd = torch.empty(m, F, dtype=torch.bfloat16, device=dev)
    us = t_us(lambda: [L._shuffled_call(xd, gus[nxt()][e], None, None, "silu", yd, cfg) for e in range(E)])
    r["gu_dense_equiv_us"] = round(us, 1)
    r["gu_dense_cfg"] = list(cfg)
    rows.append(r)
    print(json.dumps(r), flush=True)
  if args.json:
    json.dump(rows, open(args.json, "w"), indent=1)


if __name__ == "__main__":
  main()

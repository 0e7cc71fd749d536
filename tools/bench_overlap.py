"""Can decode attention (HBM-bound, below the board power cap) overlap the projection GEMMs (at the cap)?

The headline decode step is power-bound in its GEMMs (1.39 kW at 2.1 GHz, profiles/r4/power/) and HBM-bound
in attention (~0.9 kW).  A KV-head-group pipeline inside a layer would run group g's attention beside group
g+1's QKV columns / group g-1's o-projection K slice -- no weight byte read twice.  This times the pieces of
one Llama-3-70B layer at 512 sequences (half the heads = one group) alone, back to back on one stream, and as
two branches of one HIP graph (attention || QKV half + o half), replayed 20 times.

  python tools/bench_overlap.py [--json out.json]
"""
import argparse
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from xotorch_support_jetson_amd.ops import kernels as K  # noqa: E402
from xotorch_support_jetson_amd.ops.linear import linear  # noqa: E402
from xotorch_support_jetson_amd.ops.weights_layout import shuffle_for_stream  # noqa: E402


NCP = 6  # weight copies: every unit of a graph reads its own (HBM-cold, as every layer's weights are)


def graph_ms(branches, reps=5):
  """Time (ms) per unit of a graph of NCP units; in each unit the branches (lists of callables taking the unit
  index) run on separate streams and join before the next unit."""
  side = [torch.cuda.Stream() for _ in branches[1:]]
  for fns in branches:  # warm up (tuning, workspaces) outside the capture
    for f in fns:
      f(0)
  torch.cuda.synchronize()
  g = torch.cuda.CUDAGraph()
  with torch.cuda.graph(g):
    main = torch.cuda.current_stream()  # the capture stream
    streams = [main] + side
    for i in range(NCP):
      fork = torch.cuda.Event()
      fork.record(main)
      joins = []
      for s, fns in zip(streams, branches):
        s.wait_event(fork)
        with torch.cuda.stream(s):
          for f in fns:
            f(i)
          e = torch.cuda.Event()
          e.record(s)
          joins.append(e)
      for e in joins[1:]:
        main.wait_event(e)
  g.replay()
  torch.cuda.synchronize()
  st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
  best = float("inf")
  for _ in range(3):
    st.record()
    for _ in range(reps):
      g.replay()
    en.record()
    en.synchronize()
    best = min(best, st.elapsed_time(en) / reps / NCP)
  return best


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument("--json", default=None)
  args = ap.parse_args()
  dev = torch.device("cuda:0")
  torch.manual_seed(0)
  B, H, Hkv, Dh, ctx, D = 512, 64, 8, 128, 531, 8192
  Hg, Hkvg = H // 2, Hkv // 2  # one KV-head group
  pages = -(-ctx // 64)
  npool = B * pages + 4
  kc = torch.randn(npool, Hkvg, 64, Dh, device=dev).to(torch.bfloat16)
  vc = torch.randn(npool, Hkvg, Dh, 64, device=dev).to(torch.bfloat16)
  bt = torch.arange(B * pages, device=dev, dtype=torch.int32).view(B, pages).contiguous()
  cl = torch.full((B,), ctx, device=dev, dtype=torch.int32)
  q = torch.randn(B, Hg, Dh, device=dev).to(torch.bfloat16)
  ao = torch.empty_like(q)
  ws = K.DecodeWorkspace(B, Hg, Dh, pages * 64, dev)
  # weights rotated over copies (HBM-cold per call, as every layer's are)
  ncp = NCP
  wq = [shuffle_for_stream((torch.randn((Hg + 2 * Hkvg) * Dh, D, device=dev) * 0.02).to(torch.bfloat16)) for _ in range(ncp)]
  wo = [shuffle_for_stream((torch.randn(D, Hg * Dh, device=dev) * 0.02).to(torch.bfloat16)) for _ in range(ncp)]
  for w in wq + wo:
    w.xot_layout = "stream"
  x = torch.randn(B, D, device=dev).to(torch.bfloat16)
  a = torch.randn(B, Hg * Dh, device=dev).to(torch.bfloat16)
  yq = torch.empty(B, wq[0].shape[0], device=dev, dtype=torch.bfloat16)
  yo = torch.empty(B, D, device=dev, dtype=torch.bfloat16)

  wss = {a: K.DecodeWorkspace(B, Hg, Dh, pages * 64, dev, algo=a) for a in (2, 5)}
  algo = [2]

  def attn(i):
    K.attn_decode(q, kc, vc, bt, cl, 1 / math.sqrt(Dh), wss[algo[0]], ao)

  def qkv(i):
    linear(x, wq[i], out=yq)

  def oproj(i):
    linear(a, wo[i], out=yo)

  res = {"gemms_ms": graph_ms([[qkv, oproj]])}
  # (round 4 also capped the attention grid to a subset of the CUs -- XOT_ATTN_CUS, since removed: attention
  # then slows in proportion, profiles/r4/overlap/)
  for al in (2, 5):
    algo[0] = al
    for cus in (0,):
      t_a = graph_ms([[attn]])
      t_s = graph_ms([[attn, qkv, oproj]])
      t_p = graph_ms([[attn], [qkv, oproj]])
      r = dict(algo=al, attn_cus=cus or 256, attn_ms=round(t_a, 4), sequential_ms=round(t_s, 4),
               parallel_ms=round(t_p, 4), gain_pct=round(100 * (1 - t_p / t_s), 1))
      res[f"a{al}_cus{cus or 256}"] = r
      print(json.dumps(r), flush=True)
  print(json.dumps(res), flush=True)
  if args.json:
    with open(args.json, "w") as f:
      json.dump(res, f, indent=1)


if __name__ == "__main__":
  main()

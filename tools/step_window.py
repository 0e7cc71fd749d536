#!/usr/bin/env python3
"""One steady-state training step out of a rocprofv3 kernel trace: the kernels between the end of the
second-to-last optimizer burst (adamw_kernel dispatches) and the end of the last one, grouped by kernel name.
Excludes the warmup step's GEMM tuning, cache flushes and weight init that a whole-run --stats summary mixes in.

  python tools/step_window.py <trace_kernel_trace.csv> [--top 40] [--out file]"""
import argparse
import collections
import csv


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument("trace")
  ap.add_argument("--top", type=int, default=40)
  ap.add_argument("--marker", default="adamw_kernel")
  ap.add_argument("--out", default="")
  a = ap.parse_args()
  rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
  opt = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
  bursts, cur = [], [opt[0]]  # runs of marker dispatches separated by other work
  for i in opt[1:]:
    if i - cur[-1] > 50:
      bursts.append(cur)
      cur = [i]
    else:
      cur.append(i)
  bursts.append(cur)
  if len(bursts) < 2:
    raise SystemExit("need two optimizer bursts in the trace")
  lo, hi = bursts[-2][-1] + 1, bursts[-1][-1] + 1
  win = rows[lo:hi]
  t0, t1 = int(win[0]["Start_Timestamp"]), int(win[-1]["End_Timestamp"])
  agg = collections.defaultdict(lambda: [0, 0])
  for r in win:
    n = r["Kernel_Name"].split("(")[0][:120]
    agg[n][0] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    agg[n][1] += 1
  busy = sum(v[0] for v in agg.values())
  out = [f"steady-state step window: {len(win)} kernels, wall {(t1 - t0) / 1e6:.1f} ms, kernel busy {busy / 1e6:.1f} ms"]
  for n, (ns, c) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:a.top]:
    out.append(f"{ns / 1e6:8.2f} ms {100 * ns / busy:5.1f}% calls {c:5d} avg {ns / c / 1e3:8.1f} us  {n}")
  text = "\n".join(out)
  print(text)
  if a.out:
    open(a.out, "w").write(text + "\n")


if __name__ == "__main__":
  main()

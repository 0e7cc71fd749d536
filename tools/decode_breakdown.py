"""Per-kernel decode-step breakdown from a rocprofv3 kernel trace of bench.py: the window is the last
`--steps` decode rounds, delimited by the on-device sampling kernel that ends each round (so warmup
rounds with GEMM autotuning are excluded).

  python tools/decode_breakdown.py [gpurun_out/prof/<...>_kernel_trace.csv] --steps 3
"""
import argparse
import collections
import csv
import glob
import json


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument("trace", nargs="?", default=None)
  ap.add_argument("--steps", type=int, required=True, help="decode rounds in the trace (warmup + steps)")
  ap.add_argument("--json", default=None)
  a = ap.parse_args()
  path = a.trace or sorted(glob.glob("gpurun_out/prof/**/*kernel_trace.csv", recursive=True))[-1]
  rows = list(csv.DictReader(open(path)))
  ends = sorted(int(r["End_Timestamp"]) for r in rows
                if any(k in r["Kernel_Name"] for k in ("sample_kernel", "sample_stage2", "sample_fast_kernel")))
  lo, hi = ends[-(a.steps + 1)], ends[-1]
  dec = [r for r in rows if lo < int(r["Start_Timestamp"]) <= hi]
  agg = collections.defaultdict(lambda: [0, 0])
  for r in dec:
    name = r["Kernel_Name"].split("(")[0][:90]
    agg[name][0] += 1
    agg[name][1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
  tot = sum(v[1] for v in agg.values())
  span = hi - lo
  out = {"trace": path, "decode_steps": a.steps, "busy_ms_per_step": tot / a.steps / 1e6,
         "wall_ms_per_step": span / a.steps / 1e6, "kernels": []}
  for name, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    out["kernels"].append({"kernel": name, "calls_per_step": n / a.steps, "ms_per_step": t / a.steps / 1e6,
                           "pct": 100 * t / tot})
  print(f"busy {out['busy_ms_per_step']:.2f} ms/step, wall {out['wall_ms_per_step']:.2f} ms/step")
  for k in out["kernels"][:25]:
    print(f"{k['ms_per_step']:8.3f} ms {k['pct']:5.1f}%  x{k['calls_per_step']:.0f}  {k['kernel']}")
  if a.json:
    json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
  main()

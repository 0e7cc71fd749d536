"""Per-kernel time of the last K decode steps in a rocprofv3 kernel trace.  A step ends with one launch of the
sampling kernel (--marker); the window runs from the (K+1)-th last marker launch to the last, so prefill,
warmup and the GEMM policy's first-encounter timing runs stay outside.
  python tools/decode_breakdown.py gpurun_out/<dir>/trace_kernel_trace.csv --steps K [--marker NAME]"""
import argparse
import collections
import csv


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument("trace")
  ap.add_argument("--steps", type=int, required=True, help="decode steps in the traced region (warmup + timed)")
  ap.add_argument("--marker", default="sample", help="substring of the once-per-step kernel that ends a step")
  ap.add_argument("--top", type=int, default=25)
  a = ap.parse_args()
  rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
  ends = [int(r["Start_Timestamp"]) for r in rows if a.marker in r["Kernel_Name"]]
  assert len(ends) > a.steps, f"only {len(ends)} '{a.marker}' launches for {a.steps} steps"
  lo, hi = ends[-a.steps - 1], ends[-1]
  dec = [r for r in rows if lo < int(r["Start_Timestamp"]) <= hi]
  wall = (hi - lo) / 1e6 / a.steps
  tot = collections.Counter()
  calls = collections.Counter()
  for r in dec:
    n = r["Kernel_Name"].split("(")[0][:90]
    tot[n] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    calls[n] += 1
  s = sum(tot.values())
  print(f"last {a.steps} steps: {len(dec) / a.steps:.0f} kernels/step, {s / 1e6 / a.steps:.3f} ms/step busy, "
        f"{wall:.3f} ms/step wall")
  for n, t in tot.most_common(a.top):
    print(f"{t / 1e6 / a.steps:8.3f} ms/step {100 * t / s:5.1f}%  {calls[n] / a.steps:5.1f}/step  {n}")


if __name__ == "__main__":
  main()

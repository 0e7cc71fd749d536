"""Per-kernel PMC summary of a tools/gpu/pmc.sh run: the counter passes (one rocprofv3 --pmc run each) are
joined per kernel name; for every kernel whose name matches --match the last --last dispatches of each pass
are averaged, and the derived rates are computed:
  clock_ghz        GRBM_GUI_ACTIVE / 8 XCDs / dispatch time
  mfma_busy_pct    SQ_VALU_MFMA_BUSY_CYCLES / (clock cycles x 1024 SIMDs)
  td_stall_pct     TD_TC_STALL_sum / TD_TD_BUSY_sum (texture data path waiting on L2)
  l2_hit_pct       TCC_HIT / (TCC_HIT + TCC_MISS)
  fetch_gb         FETCH_SIZE (KB) x 2 (gfx950 reports half the bytes of 16-B streaming reads)
  lds_conflict_pct SQ_LDS_BANK_CONFLICT / SQ_INSTS_LDS (extra cycles per LDS instruction, %)

  python tools/pmc_summary.py gpurun_out/pmc/<name> --match gemm_big,gemm_w4,attn_decode --last 6 [--json out]
  python tools/pmc_summary.py gpurun_out/pmc/<name> --window sample_fast_kernel --last 2   (decode steps of bench.py)
"""
import argparse
import collections
import csv
import glob
import json
import os


def load_pass(d):
  files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
  per = collections.OrderedDict()  # dispatch id -> {name, grid, ns, counters}
  for f in files:
    for r in csv.DictReader(open(f)):
      did = r.get("Dispatch_Id") or r.get("Correlation_Id")
      e = per.setdefault(did, {"name": r["Kernel_Name"].split("(")[0], "grid": r.get("Grid_Size", ""), "ns": 0,
                               "start": int(r.get("Start_Timestamp", 0) or 0), "c": collections.Counter()})
      try:
        e["ns"] = max(e["ns"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
      except (KeyError, ValueError):
        pass
      e["c"][r["Counter_Name"]] += float(r["Counter_Value"])
  return per


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument("root")
  ap.add_argument("--match", default="gemm_big,gemm_w4,gemm_stream,attn_decode")
  ap.add_argument("--last", type=int, default=6)
  ap.add_argument("--json", default=None)
  ap.add_argument("--window", default=None,
                  help="kernel name that ends each step (e.g. sample_fast_kernel): only the dispatches of the last "
                       "--last steps count, grouped by (name, grid size) so tuning calls and other shapes stay out")
  a = ap.parse_args()
  pats = a.match.split(",")
  agg = collections.defaultdict(lambda: {"ns": [], "c": collections.defaultdict(list)})
  for d in sorted(glob.glob(os.path.join(a.root, "p*"))):
    if not os.path.isdir(d):
      continue
    es_all = sorted(load_pass(d).values(), key=lambda e: e["start"])
    if a.window:
      ends = [i for i, e in enumerate(es_all) if a.window in e["name"]]
      if len(ends) > a.last:
        es_all = es_all[ends[-a.last - 1] + 1:ends[-1] + 1]
    by_name = collections.defaultdict(list)
    for e in es_all:
      if any(p in e["name"] for p in pats):
        by_name[(e["name"], e["grid"]) if a.window else e["name"]].append(e)
    for key, es in by_name.items():
      for e in (es if a.window else es[-a.last:]):
        name = f"{key[0]} grid={key[1]}" if a.window else key
        agg[name]["ns"].append(e["ns"])
        for k, v in e["c"].items():
          agg[name]["c"][k].append(v)
  out = {}
  for name, g in agg.items():
    c = {k: sum(v) / len(v) for k, v in g["c"].items()}
    us = sum(g["ns"]) / len(g["ns"]) / 1e3 if g["ns"] else None
    r = {"us": round(us, 1) if us else None, "counters": {k: round(v, 1) for k, v in sorted(c.items())}}
    if "GRBM_GUI_ACTIVE" in c and us:
      cyc = c["GRBM_GUI_ACTIVE"] / 8
      r["clock_ghz"] = round(cyc / (us * 1e3), 3)
      if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
        r["mfma_busy_pct"] = round(100 * c["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * 1024), 1)
    if c.get("TD_TD_BUSY_sum"):
      r["td_stall_pct"] = round(100 * c.get("TD_TC_STALL_sum", 0) / c["TD_TD_BUSY_sum"], 1)
    if c.get("TCC_HIT_sum", 0) + c.get("TCC_MISS_sum", 0):
      r["l2_hit_pct"] = round(100 * c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"]), 1)
    if "FETCH_SIZE" in c:
      r["fetch_gb"] = round(c["FETCH_SIZE"] * 2 / 1e6, 3)
    if c.get("SQ_INSTS_LDS"):
      r["lds_conflict_pct"] = round(100 * c.get("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_INSTS_LDS"], 2)
    out[name] = r
  for name, r in sorted(out.items(), key=lambda kv: -(kv[1]["us"] or 0)):
    print(f"{r['us']:8.1f} us  mfma {r.get('mfma_busy_pct', '-'):>5}%  clk {r.get('clock_ghz', '-')}  "
          f"td-stall {r.get('td_stall_pct', '-')}%  L2 hit {r.get('l2_hit_pct', '-')}%  lds-conf {r.get('lds_conflict_pct', '-')}%  {name}")
  if a.json:
    with open(a.json, "w") as f:
      json.dump(out, f, indent=1)


if __name__ == "__main__":
  main()

"""Show or edit a persisted GEMM choice table (ops/linear.py GemmPolicy, XOT_GEMM_TABLE) -- for in-step A/Bs of one
projection's kernel choice: tune once, force one entry, run again with the same table.

  python tools/gemm_table.py show TABLE
  python tools/gemm_table.py set TABLE N K CFG_JSON [M_BUCKET]     e.g. set t.json 8192 8192 '["big", 2256, 4]'
"""
import json
import sys


def main():
  cmd, path = sys.argv[1], sys.argv[2]
  with open(path) as f:
    table = json.load(f)
  if cmd == "show":
    for k, v in sorted(table.items()):
      print(k, "->", v)
    return
  if cmd != "set":
    raise SystemExit(f"unknown command {cmd}")
  N, Kd, cfg = int(sys.argv[3]), int(sys.argv[4]), json.loads(sys.argv[5])
  mb = int(sys.argv[6]) if len(sys.argv) > 6 else None
  hit = 0
  for k in list(table):
    key = json.loads(k)
    if key[0] == "sh" and key[2] == N and key[3] == Kd and (mb is None or key[1] == mb):
      print(k, table[k], "->", cfg)
      table[k] = cfg
      hit += 1
  if not hit:
    raise SystemExit(f"no shuffled-weight entry for N={N} K={Kd}")
  with open(path, "w") as f:
    json.dump(table, f, indent=1)


if __name__ == "__main__":
  main()

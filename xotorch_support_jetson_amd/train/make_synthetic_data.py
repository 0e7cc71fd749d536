"""Generate the bundled synthetic text->SQL fine-tuning set (train 1000 / valid 100 / test 100 lines).

Deterministic (seeded): table schemas, natural-language questions and the matching SQL, in the
"table: ... columns: ... Q: ... A: SELECT ..." style.  Synthetic by construction (no dataset download).
"""
from __future__ import annotations

import json
import random
from pathlib import Path

TABLES = {
  "employees": ["name", "department", "salary", "hire_year", "city"],
  "orders": ["order_id", "customer", "amount", "status", "region"],
  "flights": ["flight_no", "origin", "destination", "duration", "carrier"],
  "books": ["title", "author", "year", "genre", "pages"],
  "matches": ["home_team", "away_team", "score", "season", "venue"],
  "gpus": ["model", "vendor", "memory_gb", "tflops", "launch_year"],
}
NUMERIC = {"salary", "hire_year", "amount", "duration", "year", "pages", "season", "memory_gb", "tflops", "launch_year"}
WORDS = ["Alpha", "Berlin", "Oslo", "Lima", "Quartz", "Nova", "Delta", "Kyoto", "Aurora", "Vega", "Rio", "Cairo"]


def example(rng: random.Random) -> str:
  table = rng.choice(list(TABLES))
  cols = TABLES[table]
  target = rng.choice(cols)
  cond = rng.choice([c for c in cols if c != target])
  if cond in NUMERIC:
    val = rng.randint(1, 2024)
    op, word = rng.choice([(">", "greater than"), ("<", "less than"), ("=", "equal to")])
    q = f"What is the {target.replace('_', ' ')} when the {cond.replace('_', ' ')} is {word} {val}?"
    sql = f"SELECT {target} FROM {table} WHERE {cond} {op} {val}"
  else:
    val = rng.choice(WORDS)
    agg = rng.choice(["", "COUNT", "MAX", "MIN"]) if target in NUMERIC else rng.choice(["", "COUNT"])
    if agg:
      q = f"What is the {agg.lower()} {target.replace('_', ' ')} for {cond.replace('_', ' ')} {val}?"
      sql = f"SELECT {agg}({target}) FROM {table} WHERE {cond} = '{val}'"
    else:
      q = f"Which {target.replace('_', ' ')} has {cond.replace('_', ' ')} {val}?"
      sql = f"SELECT {target} FROM {table} WHERE {cond} = '{val}'"
  return f"table: {table}\ncolumns: {', '.join(cols)}\nQ: {q}\nA: {sql}"


def main(out_dir: Path = Path(__file__).resolve().parent / "data" / "sql", seed: int = 7):
  rng = random.Random(seed)
  out_dir.mkdir(parents=True, exist_ok=True)
  for name, n in (("train", 1000), ("valid", 100), ("test", 100)):
    with open(out_dir / f"{name}.jsonl", "w") as f:
      for _ in range(n):
        f.write(json.dumps({"text": example(rng)}) + "\n")


if __name__ == "__main__":
  main()

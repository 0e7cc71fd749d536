"""bench.py contract: the driver's exact torchrun command line (here on CPU/gloo with a tiny model,
2 ranks) prints exactly one JSON line from rank 0 with the required keys."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _port():
  with socket.socket() as s:
    s.bind(("127.0.0.1", 0))
    return s.getsockname()[1]


@pytest.mark.parametrize("n", [1, 2])
def test_bench_json_line(n):
  args = ["bench.py", "--gpus", str(n), "--steps", "2", "--warmup", "1", "--model", "tiny-llama",
          "--batch-per-gpu", "2", "--prompt-len", "8"]
  if n == 1:
    cmd = [sys.executable] + args
  else:
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_port())] + args
  env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="2")
  r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
  assert r.returncode == 0, r.stderr[-3000:]
  lines = [l for l in r.stdout.splitlines() if l.strip().startswith("{")]
  assert len(lines) == 1, r.stdout
  d = json.loads(lines[0])
  assert KEYS <= set(d)
  assert d["n_gpus"] == n and d["steps"] == 2 and d["warmup"] == 1
  assert d["config"]["global_batch"] == 2 * n and d["value"] > 0
  assert d["scaling"] == "weak" and d["higher_is_better"] is True

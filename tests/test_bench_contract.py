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


@pytest.mark.parametrize("n", [4, 8])
def test_bench_driver_command_many_ranks(n, tmp_path):
  """The driver's exact 8-GPU command line shape (torchrun, one rank per device) at 4 and 8 ranks over gloo:
  one JSON line, weak scaling (global batch = ranks x batch per GPU), and micro-batch 0's greedy tokens equal
  the single-process run's, through the split LM head (last stage: top-k candidates of vocab rows [0, Vs);
  first stage: rows [Vs, V) + the sample)."""
  base = ["bench.py", "--steps", "3", "--warmup", "1", "--model", "tiny-llama-8l", "--batch-per-gpu", "2",
          "--prompt-len", "8", "--temperature", "0"]
  env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1")
  one = subprocess.run([sys.executable] + base + ["--gpus", "1", "--dump-tokens", str(tmp_path / "t1.json")], cwd=ROOT,
                       env=env, capture_output=True, text=True, timeout=300)
  assert one.returncode == 0, one.stderr[-3000:]
  cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}", "--master-addr",
         "127.0.0.1", "--master-port", str(_port())] + base + ["--gpus", str(n), "--dump-tokens", str(tmp_path / "tn.json")]
  r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
  assert r.returncode == 0, r.stderr[-3000:]
  lines = [l for l in r.stdout.splitlines() if l.strip().startswith("{")]
  assert len(lines) == 1, r.stdout
  d = json.loads(lines[0])
  assert d["n_gpus"] == n and d["config"]["global_batch"] == 2 * n and d["config"]["parallelism"].startswith(f"pp{n}")
  # per-rank diagnostics: one entry per rank with its layer range and bytes handed on per step
  pr = d["extra"]["per_rank"]
  assert [p["rank"] for p in pr] == list(range(n)) and all(p["send_mb_per_step"] > 0 for p in pr)
  assert pr[0]["layers"].startswith("0-") and pr[-1]["layers"].endswith("-7")
  t1, tn = json.load(open(tmp_path / "t1.json")), json.load(open(tmp_path / "tn.json"))
  # with the split head a round's ids are drawn at the start of the next round by the first stage, so the
  # ring's list starts with the prefill token and the single-process list with the first decode token
  assert tn and len(tn) == len(t1) and tn[1:] == t1[:-1]


def test_bench_more_micro_batches_than_stages(tmp_path):
  """--micro-batches 2 x world (half-size micro-batches: slack for the hop latency) keeps the node's batch and
  the tokens: sequence 0's greedy ids through a 2-rank ring of 4 one-sequence micro-batches equal the
  single-process run's, and the config reports the micro-batching."""
  base = ["bench.py", "--steps", "3", "--warmup", "1", "--model", "tiny-llama-8l", "--prompt-len", "8",
          "--temperature", "0"]
  env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1")
  one = subprocess.run([sys.executable] + base + ["--gpus", "1", "--batch-per-gpu", "2", "--dump-tokens",
                                                  str(tmp_path / "t1.json")],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
  assert one.returncode == 0, one.stderr[-3000:]
  cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
         "127.0.0.1", "--master-port", str(_port())] + base + ["--gpus", "2", "--batch-per-gpu", "2",
                                                               "--micro-batches", "4", "--dump-tokens",
                                                               str(tmp_path / "tn.json")]
  r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
  assert r.returncode == 0, r.stderr[-3000:]
  d = json.loads([l for l in r.stdout.splitlines() if l.strip().startswith("{")][-1])
  assert d["config"]["global_batch"] == 4 and d["config"]["micro_batches"] == 4
  assert d["config"]["micro_batch_size"] == 1 and "4 micro-batches x 1" in d["config"]["parallelism"]
  t1, tn = json.load(open(tmp_path / "t1.json")), json.load(open(tmp_path / "tn.json"))
  assert [s[0] for s in tn[1:]] == [s[0] for s in t1[:-1]]

"""`xot train|eval --ring`: pipeline stages as local processes over the p2p ring (gloo here, RCCL on
GPUs) with the Node path's checkpoint files and resume."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _xot(args, tmp_path, cpu=True):
  env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2", XOT_HOME=str(tmp_path / "home"))
  if cpu:
    env.update(CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
  r = subprocess.run([sys.executable, "-m", "xotorch_support_jetson_amd.main"] + args + ["--disable-tui"],
                     capture_output=True, text=True, timeout=300, env=env, cwd=str(tmp_path))
  assert r.returncode == 0, r.stderr[-3000:]
  return r.stdout


def test_ring_train_eval_resume(tmp_path):
  ds = tmp_path / "ds"
  ds.mkdir()
  for split, n in (("train", 12), ("valid", 4), ("test", 4)):
    with open(ds / f"{split}.jsonl", "w") as f:
      for i in range(n):
        f.write(json.dumps({"text": f"Q: select a from t{i}? A: SELECT a FROM t{i}"}) + "\n")
  ck = tmp_path / "ck"
  out = _xot(["train", "tiny-llama", "--ring", "--gpus", "2", "--iters", "2", "--batch-size", "4", "--micro-batch", "2",
              "--save-every", "2", "--save-checkpoint-dir", str(ck), "--data", str(ds), "--lr", "1e-3"], tmp_path)
  losses = [float(l.split("loss:")[1].split(",")[0]) for l in out.splitlines() if l.startswith("epoch")]
  assert len(losses) == 2 and losses[1] < losses[0]
  files = sorted(p.name for p in (ck / "tiny-llama").iterdir())
  assert files == ["000-001-of-004-000002.optim.safetensors", "000-001-of-004-000002.safetensors",
                   "002-003-of-004-000002.optim.safetensors", "002-003-of-004-000002.safetensors"]
  ev = _xot(["eval", "tiny-llama", "--ring", "--gpus", "2", "--batch-size", "4", "--data", str(ds),
             "--resume-checkpoint", str(ck)], tmp_path)
  assert "resumed tiny-llama from iteration 2" in ev and "eval | loss=" in ev


def test_ring_train_data_parallel(tmp_path):
  """`--parallel dp`: two full replicas, every other micro-batch each, gradients all-reduced; rank 0
  writes one full-model checkpoint that a data-parallel eval resumes from."""
  ds = tmp_path / "ds"
  ds.mkdir()
  for split, n in (("train", 12), ("valid", 4), ("test", 4)):
    with open(ds / f"{split}.jsonl", "w") as f:
      for i in range(n):
        f.write(json.dumps({"text": f"Q: select a from t{i}? A: SELECT a FROM t{i}"}) + "\n")
  ck = tmp_path / "ck"
  out = _xot(["train", "tiny-llama", "--ring", "--gpus", "2", "--parallel", "dp", "--iters", "2", "--batch-size", "4",
              "--micro-batch", "1", "--save-every", "2", "--save-checkpoint-dir", str(ck), "--data", str(ds),
              "--lr", "1e-3"], tmp_path)
  losses = [float(l.split("loss:")[1].split(",")[0]) for l in out.splitlines() if l.startswith("epoch")]
  assert len(losses) == 2 and losses[1] < losses[0]
  files = sorted(p.name for p in (ck / "tiny-llama").iterdir())
  assert files == ["000-003-of-004-000002.optim.safetensors", "000-003-of-004-000002.safetensors"]
  ev = _xot(["eval", "tiny-llama", "--ring", "--gpus", "2", "--parallel", "dp", "--batch-size", "4", "--data",
             str(ds), "--resume-checkpoint", str(ck)], tmp_path)
  assert "resumed tiny-llama from iteration 2" in ev and "eval | loss=" in ev


def test_ring_train_data_parallel_defaults_one_row_batches(tmp_path):
  """The CLI defaults (--batch-size 1 --micro-batch 1) under `--parallel dp --gpus 2`: every batch leaves
  one rank without rows; it must still join every bucket all-reduce in the same order."""
  ds = tmp_path / "ds"
  ds.mkdir()
  for split, n in (("train", 5), ("valid", 2), ("test", 3)):
    with open(ds / f"{split}.jsonl", "w") as f:
      for i in range(n):
        f.write(json.dumps({"text": f"Q: select b from u{i}? A: SELECT b FROM u{i}"}) + "\n")
  out = _xot(["train", "tiny-llama", "--ring", "--gpus", "2", "--parallel", "dp", "--iters", "2", "--data", str(ds),
              "--lr", "1e-3"], tmp_path)
  losses = [float(l.split("loss:")[1].split(",")[0]) for l in out.splitlines() if l.startswith("epoch")]
  assert len(losses) == 2 and losses[1] < losses[0]
  ev = _xot(["eval", "tiny-llama", "--ring", "--gpus", "2", "--parallel", "dp", "--data", str(ds)], tmp_path)
  assert "eval | loss=" in ev


@pytest.mark.gpu
def test_ring_train_gpu_single(gpu, tmp_path):
  """The same CLI on one MI355X (world 1: the HIP training kernels + fused AdamW)."""
  ds = tmp_path / "ds"
  ds.mkdir()
  for split, n in (("train", 8), ("valid", 2), ("test", 2)):
    with open(ds / f"{split}.jsonl", "w") as f:
      for i in range(n):
        f.write(json.dumps({"text": f"Q: select a from t{i}? A: SELECT a FROM t{i}"}) + "\n")
  out = _xot(["train", "tiny-llama", "--ring", "--gpus", "1", "--iters", "3", "--batch-size", "4", "--data", str(ds),
              "--lr", "1e-3"], tmp_path, cpu=False)
  losses = [float(l.split("loss:")[1].split(",")[0]) for l in out.splitlines() if l.startswith("epoch")]
  assert len(losses) == 3 and losses[-1] < losses[0]


def test_xot_run_gpus_defaults_to_rccl_ring(tmp_path):
  """`xot run <model> --gpus 2` (no --ring): one process per device as one ring with the p2p data plane
  (gloo on this CPU host, RCCL on GPUs) -- the same answer as the single-process run."""
  one = _xot(["run", "tiny-llama", "--prompt", "hello ring", "--max-generate-tokens", "6"], tmp_path)
  two = _xot(["run", "tiny-llama", "--gpus", "2", "--prompt", "hello ring", "--max-generate-tokens", "6"], tmp_path)
  assert "[ring 1/2]" in two and "layers 2-3" in two
  ans = lambda out: [l for l in out.splitlines() if l.strip() and not l.startswith("[")][-1]
  assert ans(two) == ans(one)


def test_ring_train_recovers_from_a_dead_stage(tmp_path):
  """3 pipeline stages; stage 1 dies in epoch 2 (XOT_FAULT=kill after 16 p2p sends: 12 per epoch).  The
  survivors detect it by heartbeat, re-form a 2-rank ring, re-partition the 4 layers over it, reload the
  epoch-1 checkpoint in process and finish the run: epochs 2 and 3 on 2 ranks, a 2-stage final checkpoint."""
  ds = tmp_path / "ds"
  ds.mkdir()
  for split, n in (("train", 12), ("valid", 4), ("test", 4)):
    with open(ds / f"{split}.jsonl", "w") as f:
      for i in range(n):
        f.write(json.dumps({"text": f"Q: select a from t{i}? A: SELECT a FROM t{i}"}) + "\n")
  ck = tmp_path / "ck"
  env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2", XOT_HOME=str(tmp_path / "home"), CUDA_VISIBLE_DEVICES="",
             HIP_VISIBLE_DEVICES="", XOT_FAULT="kill:rank=1:after=16", XOT_HEARTBEAT_TIMEOUT="3")
  r = subprocess.run([sys.executable, "-m", "xotorch_support_jetson_amd.main", "train", "tiny-llama", "--ring", "--gpus",
                      "3", "--iters", "3", "--batch-size", "4", "--micro-batch", "2", "--save-every", "1",
                      "--save-checkpoint-dir", str(ck), "--data", str(ds), "--lr", "1e-3", "--disable-tui"],
                     capture_output=True, text=True, timeout=300, env=env, cwd=str(tmp_path))
  out = r.stdout
  assert r.returncode == 0, r.stderr[-3000:] + out[-2000:]
  assert "re-forming the training ring over [0, 2]" in out and "restarting at epoch 2 on 2 rank(s)" in out
  assert "training rank 1 died (exit 17); the ring recovered without it" in out
  epochs = [l.split("|")[0].strip() for l in out.splitlines() if l.startswith("epoch")]
  assert epochs == ["epoch 1/3", "epoch 2/3", "epoch 3/3"]
  names = sorted(p.name for p in (ck / "tiny-llama").iterdir() if p.name.endswith("000003.safetensors"))
  assert names == ["000-001-of-004-000003.safetensors", "002-003-of-004-000003.safetensors"]


def test_ring_train_exit_policy():
  """run_ring: a rank that vanished (signal, injected hard exit) is what the ring recovers from; a rank that
  raised fails the run even when the survivors finished."""
  from xotorch_support_jetson_amd.train.ring_train import _peer_failure_exit
  assert _peer_failure_exit(-9) and _peer_failure_exit(17)
  assert not _peer_failure_exit(1)

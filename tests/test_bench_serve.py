"""tools/bench_serve.py --ring N measures `xot --gpus N --ring` -- the RingServer, not the single-process Node
(`xot --gpus 1` alone takes the Node path) -- and says which server answered; the server shuts down cleanly on
the SIGTERM the tool sends its process group (reference client metric: xotorch/viz/chat_tui.py:121-128)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(tmp_path, extra_env=None):
  log = tmp_path / "server.log"
  env = dict(os.environ, PYTHONPATH=ROOT, XOT_HOME=str(tmp_path / "home"), **(extra_env or {}))
  r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "bench_serve.py"), "--ring", "1", "--model",
                      "tiny-llama", "--concurrency", "4", "--max-tokens", "8", "--prompt-words", "8",
                      "--server-log", str(log)], capture_output=True, text=True, timeout=280, env=env, cwd=str(tmp_path))
  assert r.returncode == 0, r.stderr[-3000:]
  out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
  text = log.read_text()
  return out, text


def test_bench_serve_ring_measures_ring_server(tmp_path):
  out, log = _run(tmp_path, {"CUDA_VISIBLE_DEVICES": "", "HIP_VISIBLE_DEVICES": ""})
  assert out["server"] == "RingServer" and "[ring 0] ChatGPT API" in log
  assert out["output_tokens"] == 4 * 8 and out["ttft_s"]["p50"] > 0
  assert "[ring 0] exit signal: shutting down" in log and "Traceback" not in log


@pytest.mark.gpu
def test_bench_serve_ring_measures_ring_server_gpu(tmp_path):
  out, log = _run(tmp_path)
  assert out["server"] == "RingServer" and "on cuda" in log
  assert out["output_tokens"] == 4 * 8
  assert "Traceback" not in log

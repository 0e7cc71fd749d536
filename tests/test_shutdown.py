"""SIGTERM / SIGINT of a serving `xot` ends it cleanly: exit code 0, the node's tasks, discovery, gRPC server and
HTTP API shut down before the event loop closes (reference: xotorch/helpers.py:318-326, main.py:353-358)."""
import json
import os
import signal
import socket
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
  with socket.socket() as s:
    s.bind(("127.0.0.1", 0))
    return s.getsockname()[1]


@pytest.mark.parametrize("sig", [signal.SIGTERM, signal.SIGINT])
def test_xot_exits_cleanly_on_signal(tmp_path, sig):
  node_port, api_port = _port(), _port()
  cfg = tmp_path / "topology.json"
  cfg.write_text(json.dumps({"peers": {"solo": {"address": "127.0.0.1", "port": node_port, "device_capabilities": {
    "model": "t", "chip": "t", "memory": 1000, "flops": {"fp32": 1.0, "fp16": 1.0, "int8": 1.0}}}}}))
  env = dict(os.environ, XOT_HOME=str(tmp_path / "home"), PYTHONPATH=ROOT, PYTHONUNBUFFERED="1")
  out_path, err_path = tmp_path / "out.txt", tmp_path / "err.txt"
  with open(out_path, "w") as out, open(err_path, "w") as err:
    p = subprocess.Popen([sys.executable, "-m", "xotorch_support_jetson_amd.main", "--inference-engine", "dummy",
                          "--disable-tui", "--node-id", "solo", "--node-host", "127.0.0.1", "--node-port", str(node_port),
                          "--chatgpt-api-port", str(api_port), "--discovery-module", "manual",
                          "--discovery-config-path", str(cfg)], stdout=out, stderr=err, env=env, cwd=str(tmp_path))
    try:
      t_end = time.time() + 120
      while "ChatGPT API listening" not in out_path.read_text():
        assert p.poll() is None, (out_path.read_text(), err_path.read_text())
        assert time.time() < t_end, "xot did not start"
        time.sleep(0.2)
      with socket.create_connection(("127.0.0.1", api_port), timeout=5):
        pass  # the API is up
      p.send_signal(sig)
      rc = p.wait(timeout=60)
    finally:
      if p.poll() is None:
        p.kill()
  stdout, stderr = out_path.read_text(), err_path.read_text()
  assert rc == 0, (rc, stdout[-2000:], stderr[-2000:])
  assert "Received exit signal" in stdout
  assert "Event loop is closed" not in stderr and "Traceback" not in stderr, stderr[-3000:]
  with pytest.raises(OSError):  # the listener is gone
    socket.create_connection(("127.0.0.1", api_port), timeout=2).close()

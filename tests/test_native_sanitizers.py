"""Host sanitizers on the native runtime: the block manager stress test built with AddressSanitizer
and UndefinedBehaviorSanitizer (-fno-sanitize-recover) must exit cleanly.  (GPU-side sanitizers are
not available on this pool; the HIP kernels are covered by the numerics tests.)"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RT = os.path.join(ROOT, "xotorch_support_jetson_amd", "csrc", "runtime")


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
def test_block_manager_asan_ubsan(tmp_path):
  exe = tmp_path / "bm_test"
  build = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=all", "-I", RT, os.path.join(RT, "test_block_manager.cpp"), "-o", str(exe)]
  subprocess.run(build, check=True, capture_output=True, timeout=300)
  env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
  env.pop("LD_PRELOAD", None)
  r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=env)
  assert r.returncode == 0, r.stdout + r.stderr
  assert "ok" in r.stdout


def test_native_binding_invariants():
  pytest.importorskip("torch")
  try:
    from xotorch_support_jetson_amd import _runtime
  except ImportError:
    pytest.skip("native runtime not built")
  import numpy as np
  bm = _runtime.BlockManager(32, 64)
  bm.append("a", 130)
  bm.fork("a", "b", 130)
  bm.append("b", 5)
  assert bm.check()
  t = np.zeros((2, 8), dtype=np.int32)
  c = np.zeros(2, dtype=np.int32)
  bm.fill_batch(["a", "b"], t, c)
  assert list(c) == [130, 133] and t[0, 0] == t[1, 0]
  bm.free("a")
  bm.free("b")
  assert bm.num_free == 32 and bm.check()

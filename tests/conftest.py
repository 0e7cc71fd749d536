import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
  sys.path.insert(0, ROOT)


def pytest_configure(config):
  config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP kernels / RCCL)")
  config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def gpu():
  import torch
  if not torch.cuda.is_available():
    pytest.skip("no GPU")
  from xotorch_support_jetson_amd.ops._ext import require
  require()  # GPU tests must exercise the native library, never a fallback
  return torch.device("cuda:0")

"""Loader for the in-tree gfx950 kernel library (`xotorch_support_jetson_amd/_C*.so`).

On a machine with a GPU the extension MUST load: a missing or stale build raises instead of
silently falling back to eager PyTorch.  On a CPU-only host (tests, the CPU plumbing config of
BASELINE.json) `C` is None and callers use the torch reference path in `ops.reference`.
"""
from __future__ import annotations

import importlib
import os

import torch

C = None
_err: Exception | None = None
try:
  C = importlib.import_module("xotorch_support_jetson_amd._C")
except Exception as e:  # pragma: no cover - depends on the build
  _err = e


def gpu_available() -> bool:
  return torch.cuda.is_available()


def require() :
  """Return the kernel module or raise loudly (used on every GPU code path)."""
  if C is None:
    raise RuntimeError(
      "xot HIP kernel library is not built/importable "
      f"({_err!r}); run `python setup.py build_ext --inplace` (PYTORCH_ROCM_ARCH=gfx950)")
  return C


def library_path() -> str | None:
  return getattr(C, "__file__", None)


def use_kernels(device: torch.device | str | None = None) -> bool:
  """True when tensors on `device` go through the HIP kernels (every GPU device)."""
  if device is None:
    return gpu_available()
  dev = torch.device(device)
  if dev.type == "cuda":
    require()
    return True
  return False


if os.environ.get("XOT_REQUIRE_KERNELS", "0") == "1":  # pragma: no cover
  require()

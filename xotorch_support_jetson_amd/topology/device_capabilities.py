"""Per-peer device capabilities (reference: xotorch/topology/device_capabilities.py).

Differences by design: every GPU is its own peer (the reference sums all GPUs of a host into one
node and then computes on cuda:0 only, device_capabilities.py:206-316 / sharded_inference_engine.py:60-61),
and the FLOPS table knows the AMD Instinct parts (dense, non-sparse numbers).
"""
from __future__ import annotations

import os
import platform
from typing import Dict, List

import psutil
from pydantic import BaseModel


class DeviceFlops(BaseModel):
  fp32: float  # TFLOPS
  fp16: float
  int8: float

  def __str__(self):
    return f"fp32: {self.fp32:.2f} TFLOPS, fp16: {self.fp16:.2f} TFLOPS, int8: {self.int8:.2f} TFLOPS"

  def to_dict(self):
    return self.model_dump()


class DeviceCapabilities(BaseModel):
  model: str
  chip: str
  memory: int  # MB
  flops: DeviceFlops

  def __str__(self):
    return f"Model: {self.model}. Chip: {self.chip}. Memory: {self.memory}MB. Flops: {self.flops}"

  def model_post_init(self, __context) -> None:
    if isinstance(self.flops, dict):
      self.flops = DeviceFlops(**self.flops)

  def to_dict(self):
    return {"model": self.model, "chip": self.chip, "memory": self.memory, "flops": self.flops.to_dict()}


UNKNOWN_DEVICE_CAPABILITIES = DeviceCapabilities(model="Unknown Model", chip="Unknown Chip", memory=0,
                                                 flops=DeviceFlops(fp32=0, fp16=0, int8=0))

TFLOPS = 1.0
# dense (no 2:1 sparsity) vendor figures
CHIP_FLOPS: Dict[str, DeviceFlops] = {
  "AMD Instinct MI355X": DeviceFlops(fp32=157.3, fp16=2516.6, int8=5033.2),
  "AMD Instinct MI350X": DeviceFlops(fp32=144.2, fp16=2307.0, int8=4614.0),
  "AMD Instinct MI325X": DeviceFlops(fp32=163.4, fp16=1307.4, int8=2614.9),
  "AMD Instinct MI300X": DeviceFlops(fp32=163.4, fp16=1307.4, int8=2614.9),
  "AMD Instinct MI250X": DeviceFlops(fp32=47.9, fp16=383.0, int8=383.0),
  "AMD Radeon RX 7900 XTX": DeviceFlops(fp32=61.4, fp16=122.8, int8=122.8),
  "NVIDIA H100 80GB HBM3": DeviceFlops(fp32=67.0, fp16=989.0, int8=1979.0),
  "NVIDIA A100-SXM4-80GB": DeviceFlops(fp32=19.5, fp16=312.0, int8=624.0),
  "NVIDIA GEFORCE RTX 3060": DeviceFlops(fp32=13.0, fp16=26.0, int8=52.0),
  "NVIDIA JETSON AGX ORIN 32GB": DeviceFlops(fp32=17.65, fp16=35.3, int8=70.6),
}
GFX_TO_NAME = {"gfx950": "AMD Instinct MI355X", "gfx942": "AMD Instinct MI300X", "gfx90a": "AMD Instinct MI250X"}


def _lookup_flops(name: str) -> DeviceFlops:
  up = name.upper()
  for k, v in CHIP_FLOPS.items():
    if k.upper() in up or up in k.upper():
      return v
  return DeviceFlops(fp32=0, fp16=0, int8=0)


def gpu_capabilities() -> List[DeviceCapabilities]:
  """One entry per visible GPU (each GPU is a pipeline peer)."""
  import torch
  out = []
  if not torch.cuda.is_available():
    return out
  for i in range(torch.cuda.device_count()):
    p = torch.cuda.get_device_properties(i)
    arch = getattr(p, "gcnArchName", "").split(":")[0]
    name = GFX_TO_NAME.get(arch, p.name or arch or "GPU")
    out.append(DeviceCapabilities(model=f"{name} #{i}", chip=name, memory=p.total_memory // (1 << 20),
                                  flops=_lookup_flops(name)))
  return out


def cpu_capabilities() -> DeviceCapabilities:
  mem = psutil.virtual_memory().total // (1 << 20)
  return DeviceCapabilities(model=f"{platform.system()} CPU", chip=platform.processor() or platform.machine(),
                            memory=mem, flops=DeviceFlops(fp32=0, fp16=0, int8=0))


def device_capabilities(local_gpu: int | None = None) -> DeviceCapabilities:
  """Capabilities of this peer: one GPU (local_gpu or LOCAL_RANK) or the CPU when there is none."""
  try:
    gpus = gpu_capabilities()
  except Exception:
    gpus = []
  if gpus:
    idx = local_gpu if local_gpu is not None else int(os.environ.get("LOCAL_RANK", 0))
    return gpus[min(idx, len(gpus) - 1)]
  return cpu_capabilities()

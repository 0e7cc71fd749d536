"""Per-peer device capabilities (reference: xotorch/topology/device_capabilities.py).

Differences by design: every GPU is its own peer (the reference sums all GPUs of a host into one
node and then computes on cuda:0 only, device_capabilities.py:206-316 / sharded_inference_engine.py:60-61),
and the FLOPS table knows the AMD Instinct parts (dense, non-sparse numbers).
"""
from __future__ import annotations

import json
import os
import platform
import re
import subprocess
from typing import Dict, List, Optional

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
  "NVIDIA GEFORCE RTX 3090": DeviceFlops(fp32=35.6, fp16=71.0, int8=284.0),
  "NVIDIA GEFORCE RTX 4090": DeviceFlops(fp32=82.6, fp16=165.2, int8=660.6),
  "NVIDIA L40S": DeviceFlops(fp32=91.6, fp16=362.0, int8=733.0),
  "NVIDIA H200": DeviceFlops(fp32=67.0, fp16=989.0, int8=1979.0),
  "NVIDIA T1000": DeviceFlops(fp32=2.5, fp16=5.0, int8=10.0),
  "NVIDIA QUADRO M2000": DeviceFlops(fp32=1.8, fp16=0.03, int8=0.0),
  "NVIDIA QUADRO P400": DeviceFlops(fp32=0.64, fp16=0.01, int8=2.5),
  # Jetson (unified memory; the reference's home platform)
  "NVIDIA JETSON AGX ORIN 64GB": DeviceFlops(fp32=5.3, fp16=10.6, int8=275.0),
  "NVIDIA JETSON AGX ORIN 32GB": DeviceFlops(fp32=17.65, fp16=35.3, int8=70.6),
  "NVIDIA JETSON ORIN NX 16GB": DeviceFlops(fp32=1.9, fp16=3.8, int8=100.0),
  "NVIDIA JETSON ORIN NANO": DeviceFlops(fp32=1.3, fp16=2.6, int8=40.0),
  # Apple silicon (GPU)
  "Apple M1": DeviceFlops(fp32=2.29, fp16=4.58, int8=9.16),
  "Apple M1 Max": DeviceFlops(fp32=10.6, fp16=21.2, int8=42.4),
  "Apple M2": DeviceFlops(fp32=3.55, fp16=7.1, int8=14.2),
  "Apple M2 Ultra": DeviceFlops(fp32=27.2, fp16=54.4, int8=108.8),
  "Apple M3 Max": DeviceFlops(fp32=14.2, fp16=28.4, int8=56.8),
  "Apple M4": DeviceFlops(fp32=4.26, fp16=8.52, int8=17.0),
  "Apple M4 Max": DeviceFlops(fp32=18.4, fp16=36.8, int8=73.6),
  # AMD client GPUs
  "AMD Radeon RX 7900 XT": DeviceFlops(fp32=51.6, fp16=103.2, int8=103.2),
  "AMD Radeon PRO W7900": DeviceFlops(fp32=61.3, fp16=122.6, int8=122.6),
}
GFX_TO_NAME = {"gfx950": "AMD Instinct MI355X", "gfx942": "AMD Instinct MI300X", "gfx90a": "AMD Instinct MI250X"}


def _lookup_flops(name: str) -> DeviceFlops:
  """Longest table key contained in the name (so 'Apple M1 Max' is not read as 'Apple M1')."""
  up = name.upper()
  best = None
  for k, v in CHIP_FLOPS.items():
    if k.upper() in up and (best is None or len(k) > len(best[0])):
      best = (k, v)
  if best is None:
    for k, v in CHIP_FLOPS.items():
      if up and up in k.upper():
        return v
  return best[1] if best else DeviceFlops(fp32=0, fp16=0, int8=0)


# ---------------------------------------------------------------------- probes without a torch GPU
def _run(cmd: List[str], timeout: float = 10.0) -> Optional[str]:
  try:
    return subprocess.check_output(cmd, stderr=subprocess.DEVNULL, timeout=timeout).decode(errors="replace")
  except Exception:
    return None


def amd_smi_capabilities(runner=_run) -> List[DeviceCapabilities]:
  """AMD GPUs from `amd-smi static --json` (ROCm 6+) or `rocm-smi --json` when torch sees no GPU (the
  reference falls back to pyamdgpuinfo, device_capabilities.py:318-336)."""
  out = []
  txt = runner(["amd-smi", "static", "--asic", "--vram", "--json"])
  if txt:
    try:
      data = json.loads(txt)
      data = data.get("gpu_data", data) if isinstance(data, dict) else data
      for i, g in enumerate(data if isinstance(data, list) else []):
        name = (g.get("asic") or {}).get("market_name") or "AMD GPU"
        vram = (g.get("vram") or {}).get("size") or {}
        mb = int(vram.get("value", 0)) if isinstance(vram, dict) else int(str(vram).split()[0] or 0)
        out.append(DeviceCapabilities(model=f"{name} #{i}", chip=name, memory=mb, flops=_lookup_flops(name)))
    except Exception:
      out = []
  if out:
    return out
  txt = runner(["rocm-smi", "--showproductname", "--showmeminfo", "vram", "--json"])
  if txt:
    try:
      data = json.loads(txt)
      for i, (card, g) in enumerate(sorted(data.items())):
        if not card.startswith("card"):
          continue
        name = g.get("Card Series") or g.get("Card series") or g.get("Card Model") or "AMD GPU"
        total = int(g.get("VRAM Total Memory (B)", 0))
        out.append(DeviceCapabilities(model=f"{name} #{i}", chip=name, memory=total // (1 << 20),
                                      flops=_lookup_flops(name)))
    except Exception:
      out = []
  return out


def jetson_capabilities(model_path: str = "/proc/device-tree/model",
                        meminfo_path: str = "/proc/meminfo") -> Optional[DeviceCapabilities]:
  """NVIDIA Jetson: the device-tree model names the module; GPU and CPU share DRAM, so the usable memory
  is MemTotal (the reference's get_jetson_device_meminfo, device_capabilities.py:181-204)."""
  try:
    with open(model_path, "rb") as f:
      model = f.read().decode(errors="replace").strip("\x00 \n")
  except OSError:
    return None
  if "jetson" not in model.lower():
    return None
  mem_kb = 0
  try:
    with open(meminfo_path) as f:
      for line in f:
        if line.startswith("MemTotal:"):
          mem_kb = int(re.search(r"\d+", line).group())
          break
  except OSError:
    pass
  chip = model if model.upper().startswith("NVIDIA") else f"NVIDIA {model}"
  return DeviceCapabilities(model=model, chip=chip, memory=mem_kb // 1024, flops=_lookup_flops(chip))


def mac_capabilities(runner=_run) -> Optional[DeviceCapabilities]:
  """macOS: `system_profiler SPHardwareDataType` (model name, chip, memory), as the reference
  (device_capabilities.py:338-346)."""
  txt = runner(["system_profiler", "SPHardwareDataType"])
  if not txt:
    return None
  fields = {}
  for line in txt.splitlines():
    if ":" in line:
      k, v = line.split(":", 1)
      fields[k.strip()] = v.strip()
  model = fields.get("Model Name", "Mac")
  chip = fields.get("Chip", "Unknown Chip")
  mem = fields.get("Memory", "0 GB").split()
  mb = int(float(mem[0]) * (1024 if mem[1].upper().startswith("G") else 1)) if len(mem) >= 2 else 0
  return DeviceCapabilities(model=model, chip=chip, memory=mb, flops=_lookup_flops(chip))


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
  """Capabilities of this peer: one GPU (local_gpu or LOCAL_RANK) seen by torch; else a Jetson module,
  a Mac, or AMD GPUs reported by amd-smi / rocm-smi; else the CPU."""
  try:
    gpus = gpu_capabilities()
  except Exception:
    gpus = []
  idx = local_gpu if local_gpu is not None else int(os.environ.get("LOCAL_RANK", 0))
  if gpus:
    return gpus[min(idx, len(gpus) - 1)]
  if psutil.LINUX:
    j = jetson_capabilities()
    if j is not None:
      return j
  if psutil.MACOS:
    m = mac_capabilities()
    if m is not None:
      return m
  amd = amd_smi_capabilities() if psutil.LINUX else []
  if amd:
    return amd[min(idx, len(amd) - 1)]
  return cpu_capabilities()

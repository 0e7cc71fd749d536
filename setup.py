"""Build/install for the MI355X-native xot runtime.

`python setup.py build_ext --inplace` compiles the gfx950 kernel library
(`xotorch_support_jetson_amd/_C*.so`: every csrc/*.hip compiled by hipcc directly — no hipify pass,
the sources are HIP already) and the native host runtime (`xotorch_support_jetson_amd/_runtime*.so`,
C++17 + pybind11) in-tree, so the built objects travel with the repository snapshot to the GPU box.
Console script: `xot`.  (Packaging parity: reference setup.py:155-163.)
"""
import glob
import os
import shlex
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor

from setuptools import Extension, find_packages, setup
from setuptools.command.build_ext import build_ext

PKG = "xotorch_support_jetson_amd"
HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


class HipExtension(Extension):
  """Marker: sources are HIP translation units compiled with hipcc for gfx950 and linked with torch."""


class HipBuildExt(build_ext):
  def build_extension(self, ext):
    if not isinstance(ext, HipExtension):
      return super().build_extension(ext)
    import torch
    from torch.utils import cpp_extension as ce
    out = self.get_ext_fullpath(ext.name)
    os.makedirs(os.path.dirname(out), exist_ok=True)
    tmp = os.path.join(self.build_temp, ext.name.replace(".", "_"))
    os.makedirs(tmp, exist_ok=True)
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    inc = ce.include_paths(device_type="cuda") + [sysconfig.get_paths()["include"], os.path.join(HERE, CSRC)]
    cflags = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-fgpu-flush-denormals-to-zero",
              "-munsafe-fp-atomics", f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DTORCH_API_INCLUDE_EXTENSION_H",
              f"-DTORCH_EXTENSION_NAME={ext.name.split('.')[-1]}", "-DUSE_ROCM=1", "-Wno-unused-result"]
    cflags += [f"-I{p}" for p in inc]
    objs, jobs = [], []
    for src in ext.sources:
      obj = os.path.join(tmp, os.path.basename(src) + ".o")
      objs.append(obj)
      deps = [src] + glob.glob(os.path.join(CSRC, "*.h"))
      if self.force or not os.path.exists(obj) or os.path.getmtime(obj) < max(os.path.getmtime(d) for d in deps):
        jobs.append([HIPCC, "-c", src, "-o", obj] + cflags)

    def run(cmd):
      print(" ".join(shlex.quote(c) for c in cmd[:4]), flush=True)
      subprocess.run(cmd, check=True)

    with ThreadPoolExecutor(max_workers=int(os.environ.get("MAX_JOBS", "8"))) as ex:
      list(ex.map(run, jobs))
    libs = ["c10", "torch", "torch_cpu", "torch_python", "c10_hip", "torch_hip", "amdhip64"]
    ldirs = ce.library_paths(device_type="cuda")
    link = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", out] + objs + \
           [f"-L{d}" for d in ldirs] + [f"-Wl,-rpath,{d}" for d in ldirs] + [f"-l{l}" for l in libs]
    run(link)


def ext_modules():
  import pybind11
  kernels = HipExtension(name=f"{PKG}._C", sources=sorted(glob.glob(os.path.join(CSRC, "*.hip"))))
  runtime = Extension(  # plain C++17 + pybind11: no torch or HIP dependency on the host runtime
    name=f"{PKG}._runtime",
    sources=sorted(f for f in glob.glob(os.path.join(CSRC, "runtime", "*.cpp"))
                   if not os.path.basename(f).startswith("test_")),
    include_dirs=[pybind11.get_include(), os.path.join(HERE, CSRC, "runtime")],
    extra_compile_args=["-O3", "-std=c++17", "-fvisibility=hidden"],
    language="c++",
  )
  return [kernels, runtime]


setup(
  name="xot-mi355x",
  version="0.1.0",
  description="MI355X-native peer-partitioned LLM inference/training runtime (xot)",
  packages=find_packages(include=[PKG, f"{PKG}.*"]),
  package_data={PKG: ["tinychat/*", "train/data/*/*.jsonl", "csrc/*", "csrc/runtime/*"]},
  ext_modules=ext_modules(),
  cmdclass={"build_ext": HipBuildExt},
  python_requires=">=3.10",
  install_requires=["torch", "numpy", "aiohttp", "grpcio", "protobuf", "pydantic", "rich", "safetensors", "transformers",
                    "psutil", "msgpack"],
  entry_points={"console_scripts": ["xot = xotorch_support_jetson_amd.main:run"]},
)

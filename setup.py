"""Build/install for the MI355X-native xot runtime.

`python setup.py build_ext --inplace` compiles the gfx950 kernel library
(`xotorch_support_jetson_amd/_C*.so`, HIP via hipcc) and the native host runtime
(`xotorch_support_jetson_amd/_runtime*.so`, C++17) in-tree, so the built objects travel
with the repository snapshot to the GPU box.  Console script: `xot`.
(Packaging parity: reference setup.py:155-163.)
"""
import glob
import os

from setuptools import find_packages, setup

os.environ.setdefault("PYTORCH_ROCM_ARCH", "gfx950")

PKG = "xotorch_support_jetson_amd"
HERE = os.path.dirname(os.path.abspath(__file__))


def ext_modules():
  import pybind11
  from setuptools import Extension
  from torch.utils.cpp_extension import BuildExtension, CUDAExtension
  csrc = os.path.join(PKG, "csrc")
  hip_sources = sorted(glob.glob(os.path.join(csrc, "*.hip")))
  kernels = CUDAExtension(
    name=f"{PKG}._C",
    sources=hip_sources,
    include_dirs=[os.path.join(HERE, csrc)],
    extra_compile_args={
      "cxx": ["-O3", "-std=c++17"],
      "nvcc": ["-O3", "-std=c++17", "--offload-arch=gfx950", "-fgpu-flush-denormals-to-zero", "-munsafe-fp-atomics"],
    },
  )
  runtime = Extension(  # plain C++17 + pybind11: no torch or HIP dependency on the host runtime
    name=f"{PKG}._runtime",
    sources=sorted(glob.glob(os.path.join(csrc, "runtime", "*.cpp"))),
    include_dirs=[pybind11.get_include(), os.path.join(HERE, csrc, "runtime")],
    extra_compile_args=["-O3", "-std=c++17", "-fvisibility=hidden"],
    language="c++",
  )
  return [kernels, runtime], {"build_ext": BuildExtension.with_options(use_ninja=True)}


mods, cmdclass = ext_modules()
setup(
  name="xot-mi355x",
  version="0.1.0",
  description="MI355X-native peer-partitioned LLM inference/training runtime (xot)",
  packages=find_packages(include=[PKG, f"{PKG}.*"]),
  package_data={PKG: ["tinychat/*", "train/data/*/*.jsonl", "csrc/*", "csrc/runtime/*"]},
  ext_modules=mods,
  cmdclass=cmdclass,
  python_requires=">=3.10",
  install_requires=["torch", "numpy", "aiohttp", "grpcio", "protobuf", "pydantic", "rich", "safetensors", "transformers", "psutil", "msgpack"],
  entry_points={"console_scripts": ["xot = xotorch_support_jetson_amd.main:run"]},
)

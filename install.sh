#!/usr/bin/env bash
# Install xot on an MI355X host (the reference's install.sh:1-11 creates a venv and pip-installs the package;
# here the ROCm PyTorch already in the image is used as is).
#   ./install.sh            build the gfx950 kernel library + native runtime in-tree, then install `xot`
#   ./install.sh --venv     the same inside ./.venv (created with --system-site-packages, so the ROCm torch is kept)
# Needs: ROCm (hipcc under /opt/rocm or $HIPCC), python >= 3.10 with a ROCm build of torch.  No network is used:
# the package has no runtime dependencies beyond the image's.
set -euo pipefail
cd "$(dirname "$0")"
PY=${PYTHON:-python3}
if [[ "${1:-}" == "--venv" ]]; then
  "$PY" -m venv --system-site-packages .venv
  # shellcheck disable=SC1091
  source .venv/bin/activate
  PY=python
fi
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
[[ -x "$HIPCC" ]] || { echo "install.sh: hipcc not found at $HIPCC (set HIPCC)" >&2; exit 1; }
"$PY" - <<'PYEOF'
import sys
import torch
if getattr(torch.version, "hip", None) is None:
    sys.exit("install.sh: this torch is not a ROCm build")
print(f"torch {torch.__version__} (HIP {torch.version.hip})")
PYEOF
export PYTORCH_ROCM_ARCH=${PYTORCH_ROCM_ARCH:-gfx950}
"$PY" setup.py build_ext --inplace
"$PY" -m pip install --no-deps --no-build-isolation --no-index -e .
"$PY" -c "import xotorch_support_jetson_amd as x; from xotorch_support_jetson_amd.ops._ext import require; require(); print('xot installed:', x.__file__)"
echo "run: xot --help"

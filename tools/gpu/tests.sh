#!/bin/bash
# What the driver runs at round end: the GPU test suite, then smoke().   bash tools/gpu/tests.sh [pytest -k expr]
source "$(dirname "$0")/common.sh"
K=()
[ -n "$1" ] && K=(-k "$1")
step gpu_tests 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${K[@]}"
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"

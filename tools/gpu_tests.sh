#!/bin/bash
# GPU test suite + smoke (what the driver runs at round end), each step under its own time limit.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $R/gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -5 $R/gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $R/gpurun_out/gpu_tests.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $R/gpurun_out/smoke.log 2>&1; rc=$?; tail -2 $R/gpurun_out/smoke.log; exit $rc

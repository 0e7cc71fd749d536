#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_runner_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gw_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gw_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/diag/gpu_serve_split.sh

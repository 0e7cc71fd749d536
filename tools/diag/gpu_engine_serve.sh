#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/engine_gpu_tests.log 2>&1
rc=$?; echo "engine tests rc=$rc"; tail -12 gpurun_out/engine_gpu_tests.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
bash tools/diag/gpu_serve_split.sh

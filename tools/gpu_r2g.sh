#!/bin/bash
# DeepSeek training on the GPU + serving bench (presampled tokens)
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_runner_gpu.py -k "training or fused_grad" > gpurun_out/r2g_tests.log 2>&1
rc=$?; tail -15 gpurun_out/r2g_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_serve.sh

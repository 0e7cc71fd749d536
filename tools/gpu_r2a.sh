#!/bin/bash
# round 2: new-kernel GPU tests first (MLA, DeepSeek routing/models, Phi-3), then the whole GPU suite
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_runner_gpu.py tests/test_engine_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r2a_new.log 2>&1
rc=$?; echo "new rc=$rc"; tail -5 gpurun_out/r2a_new.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2a_all.log 2>&1
rc=$?; echo "all rc=$rc"; tail -5 gpurun_out/r2a_all.log; exit $rc

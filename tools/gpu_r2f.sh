#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_runner_gpu.py::test_graph_buckets_survive_workspace_growth tests/test_engine_gpu.py::test_engine_concurrent_serving_gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r2f_t.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/r2f_t.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_serve.sh

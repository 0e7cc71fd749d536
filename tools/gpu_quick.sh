#!/bin/bash
# kernel tests touched by GEMM / attention changes, then the headline bench
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "${PYTEST_K:-gemm or attn or moe}" > gpurun_out/quick_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -eq 0 ] || { tail -30 gpurun_out/quick_tests.log; exit $rc; }
timeout -k 10 900 python -u bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep metric gpurun_out/bench.log | cut -c1-200

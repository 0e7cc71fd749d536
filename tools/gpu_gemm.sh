#!/bin/bash
# GEMM kernels on the GPU: numerics tests, then the large-M benchmark.
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "gemm or moe" > gpurun_out/gemm_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u tools/bench_gemm_big.py ${GEMM_ARGS} --json gpurun_out/bench_gemm_big.json > gpurun_out/bench_gemm_big.log 2>&1
echo "bench rc=$?"

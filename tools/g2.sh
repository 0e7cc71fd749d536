#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -k "stream or gemm" > gpurun_out/g2_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/g2_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python tools/bench_gemm_m.py --json gpurun_out/gemm_m.json --ms 128,256,512 > gpurun_out/gemm_m.log 2>&1
echo "bench rc=$?" >> gpurun_out/gemm_m.log

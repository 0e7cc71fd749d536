#!/bin/bash
# round 5: the four-wave GEMM tile -- numerics first, then tall-M timing vs the ping-pong tile and hipBLASLt
source "$(dirname "$0")/common.sh"
step r5c/w4_tests 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm_w4"
step r5c/w4_bench 400 python -u tools/bench_gemm_w4.py --shapes train8b,prefill70b,decode70b
step r5c/w4_overhead 300 python -u tools/lab/gemm_overhead.py --codes 4256,2256

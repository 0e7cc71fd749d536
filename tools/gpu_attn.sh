#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "attn" > gpurun_out/attn_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -eq 0 ] || { tail -30 gpurun_out/attn_tests.log; exit $rc; }
timeout -k 10 300 python -u tools/bench_kernels.py --attn-only > gpurun_out/bench_attn.log 2>&1
echo "bench rc=$?"; grep attn_decode gpurun_out/bench_attn.log

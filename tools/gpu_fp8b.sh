#!/bin/bash
mkdir -p gpurun_out/fp8
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_runner_gpu.py -k "fp8 or stream8" > gpurun_out/fp8/tests.log 2>&1
rc=$?; tail -3 gpurun_out/fp8/tests.log; [ $rc -eq 0 ] || { grep -B5 -A30 "Error\|assert" gpurun_out/fp8/tests.log | head -80; exit $rc; }
for m in llama-3-70b llama-3-8b; do
  for b in 1 16; do
    timeout -k 10 600 python bench.py --model $m --batch-per-gpu $b --steps 32 --warmup 4 --weight-dtype fp8 > gpurun_out/fp8/bench_${m}_b${b}_fp8_v2.log 2>&1
    rc=$?; echo "$m b$b rc=$rc $(tail -1 gpurun_out/fp8/bench_${m}_b${b}_fp8_v2.log | cut -c1-200)"; [ $rc -eq 0 ] || { tail -20 gpurun_out/fp8/bench_${m}_b${b}_fp8_v2.log; exit $rc; }
  done
done

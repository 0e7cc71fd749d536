#!/bin/bash
# round 5: four-wave tile with scalar-addressed buffer-load DMA: numerics, lab timing, tall-M shapes vs hipBLASLt
source "$(dirname "$0")/common.sh"
step r5g/w4_tests 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm_w4"
mkdir -p "$O/r5g"
for s in "4096 4096 8192" "4096 28672 4096" "8192 8192 8192"; do
  timeout -k 5 60 tools/lab/w4_base $s 20 >> "$O/r5g/lab.log" 2>&1 || { echo "lab $s rc=$?"; exit 1; }
done
cat "$O/r5g/lab.log"
step r5g/w4_bench 400 python -u tools/bench_gemm_w4.py --shapes train8b,prefill70b

#!/bin/bash
# round 5: four-wave tile with inline-asm fragment reads + explicit counted waits: numerics, lab timing, GEMM table
source "$(dirname "$0")/common.sh"
step r5n/w4_tests 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm_w4"
mkdir -p "$O/r5n"
for v in base cvis nonop base; do
  for s in "4096 4096 8192" "4096 28672 4096" "8192 8192 8192"; do
    timeout -k 5 60 tools/lab/w4_$v $s 20 >> "$O/r5n/lab.log" 2>&1 || { echo "lab $v $s rc=$?"; exit 1; }
  done
done
cat "$O/r5n/lab.log"
step r5n/w4_bench 400 python -u tools/bench_gemm_w4.py --shapes train8b,prefill70b

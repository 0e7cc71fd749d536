#!/bin/bash
mkdir -p gpurun_out
for B in 384 512; do
  timeout -k 10 700 python bench.py --steps 8 --warmup 3 --batch-per-gpu $B > gpurun_out/bench_b$B.log 2>&1
  rc=$?; echo "b$B rc=$rc" >> gpurun_out/steps.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done

#!/bin/bash
# batch-per-gpu sweep of the headline bench (one GPU); stops at the first failure
mkdir -p gpurun_out
for b in 448 576 512; do
  timeout -k 10 400 python -u bench.py --batch-per-gpu $b > gpurun_out/bsweep_$b.log 2>&1
  rc=$?; echo "b=$b rc=$rc"; grep '"metric"' gpurun_out/bsweep_$b.log | cut -c1-230; [ $rc -eq 0 ] || exit $rc
done

#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/ -q -m gpu > gpurun_out/g4_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/g4_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for cfg in "l8b_b1 --model llama-3-8b --batch-per-gpu 1 --steps 32 --warmup 4" "l70b_b1 --model llama-3-70b --batch-per-gpu 1 --steps 16 --warmup 3" "l70b_b512 --steps 8 --warmup 3"; do
  set -- $cfg; name=$1; shift
  timeout -k 10 600 python bench.py "$@" > gpurun_out/g4_$name.log 2>&1 || exit $?
done

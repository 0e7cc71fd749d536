#!/bin/bash
# BASELINE.json configs 2 and 4 on one MI355X (config 3 = bench.py default, config 5 = tools/bench_train.py)
mkdir -p gpurun_out
run() {
  local name=$1; shift
  timeout -k 10 600 python bench.py "$@" > gpurun_out/cfg_$name.log 2>&1
  local rc=$?; echo "$name rc=$rc" >> gpurun_out/steps.log
  if [ $rc -ne 0 ]; then exit $rc; fi
}
run l8b_b1 --model llama-3-8b --batch-per-gpu 1 --steps 32 --warmup 4
run l8b_b512 --model llama-3-8b --batch-per-gpu 512 --steps 16 --warmup 3
run mixtral_b1 --model mixtral-8x7b --batch-per-gpu 1 --steps 32 --warmup 4
run mixtral_b512 --model mixtral-8x7b --batch-per-gpu 512 --steps 8 --warmup 3
run l70b_b1 --model llama-3-70b --batch-per-gpu 1 --steps 16 --warmup 3
timeout -k 10 900 python tools/bench_train.py > gpurun_out/cfg_train_l8b.log 2>&1; echo "train rc=$?" >> gpurun_out/steps.log

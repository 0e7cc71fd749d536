#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 900 python tools/bench_train.py --model llama-3-8b --seq 2048 --mb 1 --microbatches 8 --steps 3 --warmup 1 > gpurun_out/train_8b.log 2>&1
echo "rc=$?" >> gpurun_out/train_8b.log

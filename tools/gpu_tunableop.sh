#!/bin/bash
mkdir -p gpurun_out
export PYTORCH_TUNABLEOP_ENABLED=1
export PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_results%d.csv
export PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=20
timeout -k 10 1000 python bench.py --steps 8 --warmup 3 > gpurun_out/bench_tunable.log 2>&1
echo "rc=$?" >> gpurun_out/bench_tunable.log

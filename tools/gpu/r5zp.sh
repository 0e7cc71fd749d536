#!/bin/bash
# round 5: fp32 GradAccs for the RMSNorm weights: numerics, training A/B
source "$(dirname "$0")/common.sh"
step r5zp/tests 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_train_own_gpu.py tests/test_engine_gpu.py tests/test_runner_gpu.py tests/test_data_parallel.py -k "embed or ragged or train or fused or grad or side or norm or head or moe or deepseek"
step r5zp/train 600 python -u tools/bench_train.py --model llama-3-8b --seq 2048 --mb 2 --microbatches 4 --steps 4 --warmup 1
XOT_NORM_ACC=0 step r5zp/train_dense 600 python -u tools/bench_train.py --model llama-3-8b --seq 2048 --mb 2 --microbatches 4 --steps 4 --warmup 1
step r5zp/train_b 600 python -u tools/bench_train.py --model llama-3-8b --seq 2048 --mb 2 --microbatches 4 --steps 4 --warmup 1

#!/bin/bash
# round 5: QKV split + RoPE in one autograd function (rope reads the qkv rows, backward writes dqkv slices)
source "$(dirname "$0")/common.sh"
step r5zk/tests 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_train_own_gpu.py tests/test_engine_gpu.py tests/test_runner_gpu.py tests/test_data_parallel.py -k "ragged or train or fused or grad or side or moe or deepseek"
step r5zk/train 600 python -u tools/bench_train.py --model llama-3-8b --seq 2048 --mb 2 --microbatches 4 --steps 4 --warmup 1
step r5zk/train_b 600 python -u tools/bench_train.py --model llama-3-8b --seq 2048 --mb 2 --microbatches 4 --steps 4 --warmup 1

#!/bin/bash
# round 5: dK / dV kernel without the P^T LDS round trip (v2): numerics, training A/B, steady-state step profile
source "$(dirname "$0")/common.sh"
step r5zb/tests 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_train_own_gpu.py -k "attention_train or deepseek_dims or ragged"
step r5zb/train_v2 600 python -u tools/bench_train.py --model llama-3-8b --seq 2048 --mb 2 --microbatches 4 --steps 4 --warmup 1
XOT_TRAIN_DKDV_V1=1 step r5zb/train_v1 600 python -u tools/bench_train.py --model llama-3-8b --seq 2048 --mb 2 --microbatches 4 --steps 4 --warmup 1
step r5zb/train_v2b 600 python -u tools/bench_train.py --model llama-3-8b --seq 2048 --mb 2 --microbatches 4 --steps 4 --warmup 1
prof r5zb/trainprof 600 python3 "$R/tools/bench_train.py" --mb 2 --microbatches 4 --steps 2 --warmup 1
step r5zb/trainstep 60 python tools/step_window.py "$(ls "$O"/r5zb/trainprof/*kernel_trace.csv | head -1)" --top 45

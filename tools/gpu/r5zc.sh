#!/bin/bash
# round 5: dQ kernel without the dS LDS round trip (v2): numerics, training A/B, steady-state step profile
source "$(dirname "$0")/common.sh"
step r5zc/tests 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_train_own_gpu.py -k "attention_train or deepseek_dims or ragged"
step r5zc/train_v2 600 python -u tools/bench_train.py --model llama-3-8b --seq 2048 --mb 2 --microbatches 4 --steps 4 --warmup 1
XOT_TRAIN_DQ_V1=1 step r5zc/train_v1 600 python -u tools/bench_train.py --model llama-3-8b --seq 2048 --mb 2 --microbatches 4 --steps 4 --warmup 1
step r5zc/train_v2b 600 python -u tools/bench_train.py --model llama-3-8b --seq 2048 --mb 2 --microbatches 4 --steps 4 --warmup 1
step r5zc/attn_v2 120 python -u tools/bench_attn_train.py
XOT_TRAIN_DQ_V1=1 step r5zc/attn_dq1 120 python -u tools/bench_attn_train.py
XOT_TRAIN_DQ_V1=1 XOT_TRAIN_DKDV_V1=1 step r5zc/attn_v1 120 python -u tools/bench_attn_train.py

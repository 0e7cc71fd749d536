#!/bin/bash
# round 5: v2-schedule training attention forward: numerics, attention microbench, train bench A/B
source "$(dirname "$0")/common.sh"
step r5j/tests 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_train_own_gpu.py tests/test_engine_gpu.py -k "attention_train or vision or train or ragged"
step r5j/train_v2 600 python -u tools/bench_train.py --model llama-3-8b --seq 2048 --mb 2 --microbatches 4 --steps 4 --warmup 1
XOT_TRAIN_ATTN_V1=1 step r5j/train_v1 600 python -u tools/bench_train.py --model llama-3-8b --seq 2048 --mb 2 --microbatches 4 --steps 4 --warmup 1

#!/bin/bash
# round 5: v2-schedule dQ pass of the training attention: numerics, training tests, train bench A/B
source "$(dirname "$0")/common.sh"
step r5r/tests 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_train_own_gpu.py tests/test_engine_gpu.py tests/test_runner_gpu.py -k "attention_train or train or ragged or grad"
step r5r/train_dq2 600 python -u tools/bench_train.py --model llama-3-8b --seq 2048 --mb 2 --microbatches 4 --steps 4 --warmup 1
XOT_TRAIN_DQ_V1=1 step r5r/train_dq1 600 python -u tools/bench_train.py --model llama-3-8b --seq 2048 --mb 2 --microbatches 4 --steps 4 --warmup 1

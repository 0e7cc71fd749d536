#!/bin/bash
# round 5: AdamW fused with the operand-layout refresh: numerics, training tests, train bench A/B
source "$(dirname "$0")/common.sh"
step r5k/tests 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_train_own_gpu.py tests/test_engine_gpu.py tests/test_runner_gpu.py -k "adamw or train or ragged"
step r5k/train_fused 600 python -u tools/bench_train.py --model llama-3-8b --seq 2048 --mb 2 --microbatches 4 --steps 4 --warmup 1
XOT_FUSED_ADAMW=0 step r5k/train_plain 600 python -u tools/bench_train.py --model llama-3-8b --seq 2048 --mb 2 --microbatches 4 --steps 4 --warmup 1
step r5k/b256 500 python -u bench.py --batch-per-gpu 256 --steps 20 --warmup 5

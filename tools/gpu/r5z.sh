#!/bin/bash
# round 5: LM head gradient into a GradAcc on the side stream: numerics, training bench A/B on one box
source "$(dirname "$0")/common.sh"
step r5z/tests 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_train_own_gpu.py tests/test_engine_gpu.py tests/test_runner_gpu.py tests/test_data_parallel.py -k "ragged or train or fused or grad or head or dp or data or side"
step r5z/train 600 python -u tools/bench_train.py --model llama-3-8b --seq 2048 --mb 2 --microbatches 4 --steps 4 --warmup 1
XOT_DW_STREAM=0 step r5z/train_dw0 600 python -u tools/bench_train.py --model llama-3-8b --seq 2048 --mb 2 --microbatches 4 --steps 4 --warmup 1
step r5z/train_b 600 python -u tools/bench_train.py --model llama-3-8b --seq 2048 --mb 2 --microbatches 4 --steps 4 --warmup 1

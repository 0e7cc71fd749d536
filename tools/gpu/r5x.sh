#!/bin/bash
# round 5: grad-norm two-level reduce: numerics + training bench
source "$(dirname "$0")/common.sh"
step r5x/tests 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_train_own_gpu.py tests/test_engine_gpu.py -k "sumsq or ragged or train"
step r5x/train 600 python -u tools/bench_train.py --model llama-3-8b --seq 2048 --mb 2 --microbatches 4 --steps 4 --warmup 1

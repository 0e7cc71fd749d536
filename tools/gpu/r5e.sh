#!/bin/bash
# round 5: four-wave tile numerics + timing after the read-order change, then training with 4256 in the tuner
source "$(dirname "$0")/common.sh"
step r5e/w4_tests 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm_w4"
step r5e/w4_bench 400 python -u tools/bench_gemm_w4.py --shapes train8b
step r5e/train_gemms 300 python -u tools/bench_train_gemms.py --tokens 4096
step r5e/train 600 python -u tools/bench_train.py --model llama-3-8b --seq 2048 --mb 2 --microbatches 4 --steps 3 --warmup 1

#!/bin/bash
# round 5: transposed-staging relayout kernels: numerics, training bench, steady-state step profile
source "$(dirname "$0")/common.sh"
step r5w/tests 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_train_own_gpu.py -k "relayout or adamw or ragged"
step r5w/train 600 python -u tools/bench_train.py --model llama-3-8b --seq 2048 --mb 2 --microbatches 4 --steps 4 --warmup 1
prof r5w/trainprof 600 python3 "$R/tools/bench_train.py" --mb 2 --microbatches 4 --steps 2 --warmup 1
step r5w/trainstep 60 python tools/step_window.py "$(ls "$O"/r5w/trainprof/*kernel_trace.csv | head -1)" --top 40

#!/bin/bash
# round 5: four-wave tile (static schedule) numerics, training bench + steady-state step profile, headline bench
source "$(dirname "$0")/common.sh"
step r5h/w4_tests 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm_w4"
step r5h/train 600 python -u tools/bench_train.py --model llama-3-8b --seq 2048 --mb 2 --microbatches 4 --steps 3 --warmup 1
prof r5h/trainprof 600 python3 "$R/tools/bench_train.py" --mb 2 --microbatches 4 --steps 2 --warmup 1
step r5h/trainstep 60 python tools/step_window.py "$(ls "$O"/r5h/trainprof/*kernel_trace.csv | head -1)" --top 40
step r5h/headline 500 python -u bench.py --steps 20 --warmup 5

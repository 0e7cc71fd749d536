#!/bin/bash
# round 5: vectorized fp32 cross-entropy kernels: numerics, training bench, step profile
source "$(dirname "$0")/common.sh"
step r5zj/tests 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_runner_gpu.py -k "cross_entropy or fused_head"
step r5zj/train 600 python -u tools/bench_train.py --model llama-3-8b --seq 2048 --mb 2 --microbatches 4 --steps 4 --warmup 1
step r5zj/train_b 600 python -u tools/bench_train.py --model llama-3-8b --seq 2048 --mb 2 --microbatches 4 --steps 4 --warmup 1
prof r5zj/trainprof 600 python3 "$R/tools/bench_train.py" --mb 2 --microbatches 4 --steps 2 --warmup 1
step r5zj/trainstep 60 python tools/step_window.py "$(ls "$O"/r5zj/trainprof/*kernel_trace.csv | head -1)" --top 45

#!/bin/bash
# round 5: steady-state training step profile with the weight-gradient side stream
source "$(dirname "$0")/common.sh"
prof r5zh/trainprof 600 python3 "$R/tools/bench_train.py" --mb 2 --microbatches 4 --steps 2 --warmup 1
step r5zh/trainstep 60 python tools/step_window.py "$(ls "$O"/r5zh/trainprof/*kernel_trace.csv | head -1)" --top 45

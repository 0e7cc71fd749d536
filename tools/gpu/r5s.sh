#!/bin/bash
# round 5: training knob sweep on one box (CE chunk rows, four-wave preference threshold, raster group)
source "$(dirname "$0")/common.sh"
T="python -u tools/bench_train.py --model llama-3-8b --seq 2048 --mb 2 --microbatches 4 --steps 4 --warmup 1"
step r5s/base 600 $T
XOT_CE_CHUNK=2048 step r5s/ce2048 600 $T
XOT_CE_CHUNK=4096 step r5s/ce4096 600 $T
XOT_GEMM_W4_PREF_M=1024 step r5s/pref1024 600 $T
XOT_GEMM_GROUP_M=8 step r5s/gm8 600 $T
step r5s/base2 600 $T

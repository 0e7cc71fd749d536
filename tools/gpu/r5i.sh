#!/bin/bash
# round 5: A/B on one box: residual join in the RMSNorm backward + multi-tensor grad norm, on vs off
source "$(dirname "$0")/common.sh"
step r5i/train_on 600 python -u tools/bench_train.py --model llama-3-8b --seq 2048 --mb 2 --microbatches 4 --steps 4 --warmup 1
XOT_RESNORM=0 XOT_MULTI_SUMSQ=0 step r5i/train_off 600 python -u tools/bench_train.py --model llama-3-8b --seq 2048 --mb 2 --microbatches 4 --steps 4 --warmup 1
step r5i/train_on2 600 python -u tools/bench_train.py --model llama-3-8b --seq 2048 --mb 2 --microbatches 4 --steps 4 --warmup 1

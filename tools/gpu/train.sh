#!/bin/bash
# Training (BASELINE config 5: Llama-3-8B, seq 2048) and its kernel profile.   bash tools/gpu/train.sh [bench|prof|mixtral]...
source "$(dirname "$0")/common.sh"
for what in ${@:-bench}; do
  case $what in
    bench)   step train/l8b 900 python tools/bench_train.py --model llama-3-8b --seq 2048 --mb 1 --microbatches 8 --steps 3 --warmup 1 ;;
    prof)    prof train/prof 900 python3 "$R/tools/bench_train.py" --steps 3 --warmup 1 ;;
    mixtral) step train/mixtral_4l 900 python tools/bench_train.py --model mixtral-8x7b --layers 4 ;;
  esac
done

#!/bin/bash
# Training (BASELINE config 5: Llama-3-8B, seq 2048) and its kernel profile.   bash tools/gpu/train.sh [bench|group|blas|prof|mixtral]...
source "$(dirname "$0")/common.sh"
for what in ${@:-bench}; do
  case $what in
    bench)   step train/l8b 900 python tools/bench_train.py --model llama-3-8b --seq 2048 --mb 2 --microbatches 4 --steps 3 --warmup 1 ;;
    group)   # grouped raster of the tall gemm_big grids: off (1) / 4 (default) / 8
             for gm in 1 8; do XOT_GEMM_GROUP_M=$gm step train/l8b_group$gm 900 python tools/bench_train.py --model llama-3-8b --seq 2048 --mb 2 --microbatches 4 --steps 3 --warmup 1; done ;;
    blas)    XOT_TRAIN_OWN_GEMM=0 step train/l8b_blas 900 python tools/bench_train.py --model llama-3-8b --seq 2048 --mb 2 --microbatches 4 --steps 3 --warmup 1 ;;
    prof)    prof train/prof 900 python3 "$R/tools/bench_train.py" --mb 2 --microbatches 4 --steps 3 --warmup 1 ;;
    mixtral) step train/mixtral_4l 900 python tools/bench_train.py --model mixtral-8x7b --layers 4 ;;
  esac
done

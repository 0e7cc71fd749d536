#!/bin/bash
# round 5: training attention backward v2 with transposed LDS reads (no transposed images): numerics, isolated timing, training A/B
source "$(dirname "$0")/common.sh"
step r5ze/tests 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_train_own_gpu.py -k "attention_train or deepseek_dims or ragged or bidir"
step r5ze/attn_v2 120 python -u tools/bench_attn_train.py
XOT_TRAIN_DQ_V1=1 XOT_TRAIN_DKDV_V1=1 step r5ze/attn_v1 120 python -u tools/bench_attn_train.py
step r5ze/attn_v2_d64 120 python -u tools/bench_attn_train.py --Dh 64 --H 32 --Hkv 8
step r5ze/train_v2 600 python -u tools/bench_train.py --model llama-3-8b --seq 2048 --mb 2 --microbatches 4 --steps 4 --warmup 1
XOT_TRAIN_DQ_V1=1 XOT_TRAIN_DKDV_V1=1 step r5ze/train_v1 600 python -u tools/bench_train.py --model llama-3-8b --seq 2048 --mb 2 --microbatches 4 --steps 4 --warmup 1
step r5ze/train_v2b 600 python -u tools/bench_train.py --model llama-3-8b --seq 2048 --mb 2 --microbatches 4 --steps 4 --warmup 1

#!/bin/bash
# round 5: SiLU backward in the down projection's dA GEMM epilogue (EPI_SILU_BWD): numerics, training A/B
source "$(dirname "$0")/common.sh"
step r5zg/tests 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_train_own_gpu.py tests/test_engine_gpu.py tests/test_kernels_gpu.py -k "silu or ragged or train or gemm_w4"
step r5zg/train_fused 600 python -u tools/bench_train.py --model llama-3-8b --seq 2048 --mb 2 --microbatches 4 --steps 4 --warmup 1
XOT_SILU_BWD_FUSED=0 step r5zg/train_plain 600 python -u tools/bench_train.py --model llama-3-8b --seq 2048 --mb 2 --microbatches 4 --steps 4 --warmup 1
step r5zg/train_fused_b 600 python -u tools/bench_train.py --model llama-3-8b --seq 2048 --mb 2 --microbatches 4 --steps 4 --warmup 1

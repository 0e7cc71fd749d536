#!/bin/bash
# round 5: two query heads per dK/dV workgroup (half the partial slabs); prefill chunk 12288 A/B
source "$(dirname "$0")/common.sh"
step r5zm/tests 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention_train or deepseek_dims"
step r5zm/attn_hpw2 120 python -u tools/bench_attn_train.py
XOT_TRAIN_DKDV_HPW=1 step r5zm/attn_hpw1 120 python -u tools/bench_attn_train.py
step r5zm/train 600 python -u tools/bench_train.py --model llama-3-8b --seq 2048 --mb 2 --microbatches 4 --steps 4 --warmup 1
step r5zm/chunk8192 500 python -u bench.py --steps 20 --warmup 5
XOT_PREFILL_CHUNK=12288 step r5zm/chunk12288 500 python -u bench.py --steps 20 --warmup 5

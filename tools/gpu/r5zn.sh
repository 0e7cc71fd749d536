#!/bin/bash
# round 5: same-box A/B: dK/dV heads per workgroup (training step), prefill chunk 8192 vs 12288 interleaved
source "$(dirname "$0")/common.sh"
step r5zn/train_hpw2 600 python -u tools/bench_train.py --model llama-3-8b --seq 2048 --mb 2 --microbatches 4 --steps 4 --warmup 1
XOT_TRAIN_DKDV_HPW=1 step r5zn/train_hpw1 600 python -u tools/bench_train.py --model llama-3-8b --seq 2048 --mb 2 --microbatches 4 --steps 4 --warmup 1
step r5zn/train_hpw2b 600 python -u tools/bench_train.py --model llama-3-8b --seq 2048 --mb 2 --microbatches 4 --steps 4 --warmup 1
step r5zn/c8192a 500 python -u bench.py --steps 10 --warmup 3
XOT_PREFILL_CHUNK=12288 step r5zn/c12288a 500 python -u bench.py --steps 10 --warmup 3
step r5zn/c8192b 500 python -u bench.py --steps 10 --warmup 3
XOT_PREFILL_CHUNK=12288 step r5zn/c12288b 500 python -u bench.py --steps 10 --warmup 3

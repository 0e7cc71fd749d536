#!/bin/bash
# round 5: headline + prefill with the untimed tall-GEMM choice, training bench
source "$(dirname "$0")/common.sh"
step r5u/headline 500 python -u bench.py --steps 20 --warmup 5
step r5u/train 600 python -u tools/bench_train.py --model llama-3-8b --seq 2048 --mb 2 --microbatches 4 --steps 4 --warmup 1
grep -h "prefill" "$O"/r5u/headline.log

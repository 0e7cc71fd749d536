#!/bin/bash
# round 5, second GPU pass: gemm_big per-tile fixed cost vs k-step cost (lab), the headline bench, and the
# RingServer at the headline operating point through the HTTP API
source "$(dirname "$0")/common.sh"
step r5b/gemm_overhead 300 python -u tools/lab/gemm_overhead.py
step r5b/bench 400 python -u bench.py --steps 20 --warmup 5
step r5b/ring70 1000 python -u tools/bench_serve.py --ring 1 --model llama-3-70b --concurrency 512 --max-tokens 128 --prompt-words 124

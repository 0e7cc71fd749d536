#!/bin/bash
# round 5: kernel trace of the headline's prefill (512 x 512 tokens) -- what besides the GEMMs takes its time
source "$(dirname "$0")/common.sh"
prof r5q/prof 900 python3 "$R/bench.py" --steps 2 --warmup 1
bash "$(dirname "$0")/pmc.sh" w4_prefill_gu python3 "$R/tools/bench_gemm_w4.py" --mnk 8192,57344,8192,silu --codes 4256 --no-blas
bash "$(dirname "$0")/pmc.sh" w4_prefill_dn python3 "$R/tools/bench_gemm_w4.py" --mnk 8192,8192,28672,resid --codes 4256 --no-blas

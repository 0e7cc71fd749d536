#!/bin/bash
# round 5: PMC passes of hipBLASLt at M = N = 4096, K = 8192 (compare with the four-wave tile's passes)
source "$(dirname "$0")/common.sh"
bash "$(dirname "$0")/pmc.sh" w4_blas python3 "$R/tools/bench_gemm_w4.py" --mnk 4096,4096,8192,none --codes none

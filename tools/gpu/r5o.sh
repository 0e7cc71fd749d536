#!/bin/bash
# round 5: decode-shape GEMMs (70B, 512 rows) four-wave vs two-phase tile per K split, then the headline bench
source "$(dirname "$0")/common.sh"
for S in 1 2 3 4; do
  step r5o/dec_s$S 300 python -u tools/bench_gemm_w4.py --shapes decode70b --splits $S
done
XOT_GEMM_TUNE_LOG=1 step r5o/headline 500 python -u bench.py --steps 20 --warmup 5

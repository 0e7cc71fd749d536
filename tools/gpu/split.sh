#!/bin/bash
# A/B of the split decode step (two half-batches on two streams, models/transformer.py:_forward_split)
# against the single-stream step at the headline config.
#   bash tools/gpu/split.sh [base|split|split0|prof]...
source "$(dirname "$0")/common.sh"
for what in ${@:-base split split0}; do
  case $what in
    base)   step split/base 400 python -u bench.py --steps 10 --warmup 3 ;;
    split)  XOT_SPLIT_DECODE=256 step split/split 400 python -u bench.py --steps 10 --warmup 3 ;;
    split0) XOT_SPLIT_DECODE=256 XOT_SPLIT_OFFSET=0 step split/split0 400 python -u bench.py --steps 10 --warmup 3 ;;
    eager)  XOT_SPLIT_DECODE=256 XOT_GRAPHS=0 step split/split_eager 400 python -u bench.py --steps 10 --warmup 3 ;;
    attnnt|wg8|slab|grp) ;;
    prof)   XOT_SPLIT_DECODE=256 prof split/prof 600 python3 "$R/bench.py" --steps 6 --warmup 3
            step split/breakdown 60 python tools/decode_breakdown.py "$(ls "$O"/split/prof/*/*kernel_trace.csv "$O"/split/prof/*kernel_trace.csv 2>/dev/null | head -1)" --steps 6 --json "$O/split/breakdown.json" ;;
  esac
done
# attnnt: decode attention with non-temporal K / V loads (XOT_ATTN_DECODE=3) against the default
if [ "$1" = attnnt ]; then
  step attnnt/test 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k attn_decode
  step attnnt/base 400 python -u bench.py --steps 10 --warmup 3
  XOT_ATTN_DECODE=3 step attnnt/nt 400 python -u bench.py --steps 10 --warmup 3
fi
# wg8: 8-wave single-partition decode attention at small batch vs the 4-wave split + merge (XOT_ATTN_WG8_PAGES=0)
if [ "$1" = wg8 ]; then
  step wg8/test 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k attn_decode tests/test_runner_gpu.py tests/test_split_decode_gpu.py
  step wg8/b1_new 300 python -u bench.py --model llama-3-8b --batch-per-gpu 1 --steps 32 --warmup 4
  XOT_ATTN_WG8_PAGES=0 step wg8/b1_old 300 python -u bench.py --model llama-3-8b --batch-per-gpu 1 --steps 32 --warmup 4
  step wg8/b1_new2 300 python -u bench.py --model llama-3-8b --batch-per-gpu 1 --steps 32 --warmup 4
  step wg8/b1_70b 400 python -u bench.py --model llama-3-70b --batch-per-gpu 1 --steps 16 --warmup 3
fi
# slab: GEMM tuner charging the split-K slab read-back (default) vs GEMM time only
if [ "$1" = slab ]; then
  XOT_HOME=$O/slab/home_new step slab/new 400 python -u bench.py --steps 10 --warmup 3
  XOT_SLAB_TBPS=0 XOT_HOME=$O/slab/home_old step slab/old 400 python -u bench.py --steps 10 --warmup 3
  XOT_HOME=$O/slab/home_new step slab/new_again 400 python -u bench.py --steps 10 --warmup 3
fi
# grp: grouped raster of tall gemm_big grids -- kernel tests, GEMM shapes at prefill M, headline prefill time
if [ "$1" = grp ]; then
  step grp/test 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm_big or moe"
  step grp/gemm 500 python -u tools/bench_gemm_sk.py --ms 2048,8192 --json "$O/grp/gemm.json"
  step grp/headline 400 python -u bench.py --steps 10 --warmup 3
fi

#!/bin/bash
# Headline (BASELINE config 3, Llama-3-70B, 512 sequences, one GPU) and its kernel breakdown.
#   bash tools/gpu/headline.sh [bench|ab|sk|tune|pp2|prof|sweep]...      (default: bench prof)
source "$(dirname "$0")/common.sh"
for what in ${@:-bench prof}; do
  case $what in
    bench) step headline/bench 400 python -u bench.py --steps 20 --warmup 5 ;;
    ab)    # own kernels for every projection vs gate/up row-major on hipBLASLt
           step headline/own 400 python -u bench.py --steps 10 --warmup 3
           XOT_ROWMAJOR_PROJ=gu step headline/gu_hipblaslt 400 python -u bench.py --steps 10 --warmup 3 ;;
    prof)  prof headline/prof 600 python3 "$R/bench.py" --steps 6 --warmup 3
           step headline/breakdown 60 python tools/decode_breakdown.py "$(ls "$O"/headline/prof/*/*kernel_trace.csv "$O"/headline/prof/*kernel_trace.csv 2>/dev/null | head -1)" --steps 6 --json "$O/headline/breakdown.json"
           cat "$O/headline/breakdown.log" ;;
    sk)    # stream-K in the tuner's candidates or not (the tuner times short bursts; the step runs at the power cap)
           XOT_GEMM_TABLE=$O/headline/tbl_default.json step headline/sk_on 400 python -u bench.py --steps 20 --warmup 5
           XOT_GEMM_SK=0 XOT_GEMM_TABLE=$O/headline/tbl_nosk.json step headline/sk_off 400 python -u bench.py --steps 20 --warmup 5
           XOT_GEMM_TABLE=$O/headline/tbl_default.json step headline/sk_on2 400 python -u bench.py --steps 20 --warmup 5 ;;
    tune)  # GEMM tuner timing at the power cap (sustained, default) vs isolated cold calls (XOT_TUNE_SUSTAINED_M=0)
           XOT_GEMM_TABLE=$O/headline/tbl_sustained.json step headline/tune_sustained 600 python -u bench.py --steps 20 --warmup 5
           XOT_TUNE_SUSTAINED_M=0 XOT_GEMM_TABLE=$O/headline/tbl_isolated.json step headline/tune_isolated 400 python -u bench.py --steps 20 --warmup 5
           XOT_GEMM_TABLE=$O/headline/tbl_sustained.json step headline/tune_sustained2 400 python -u bench.py --steps 20 --warmup 5 ;;
    pp2)   # two-phase ping-pong tile offered (default) vs not, same box
           XOT_GEMM_TABLE=$O/headline/tbl_pp2.json step headline/pp2_on 400 python -u bench.py --steps 20 --warmup 5
           XOT_GEMM_PP2=0 XOT_GEMM_TABLE=$O/headline/tbl_nopp2.json step headline/pp2_off 400 python -u bench.py --steps 20 --warmup 5
           XOT_GEMM_TABLE=$O/headline/tbl_pp2.json step headline/pp2_on2 400 python -u bench.py --steps 20 --warmup 5 ;;
    sweep) for b in 448 512 576; do step headline/b$b 400 python -u bench.py --batch-per-gpu $b --steps 10 --warmup 3; done ;;
  esac
done

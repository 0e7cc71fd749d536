#!/bin/bash
# Headline (BASELINE config 3, Llama-3-70B, 512 sequences, one GPU) and its kernel breakdown.
#   bash tools/gpu/headline.sh [bench|ab|sk|tune|pp2|oproj|tunelog|tiex|b384|vtail|srr|prof|sweep]...      (default: bench prof)
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
    oproj) # o-proj (N = K = 8192) kernel choice in the step: tuned pick vs the two-phase 256 x 256 tile at S 4 / 2
           T=$O/headline/tbl_o.json
           XOT_GEMM_TABLE=$T step headline/o_tuned 400 python -u bench.py --steps 20 --warmup 5
           python tools/gemm_table.py show "$T" > "$O/headline/tbl_o_tuned.txt"
           for c in 4 2; do cp "$T" "$O/headline/tbl_o$c.json"
             python tools/gemm_table.py set "$O/headline/tbl_o$c.json" 8192 8192 "[\"big\", 2256, $c]" 512
             XOT_GEMM_TABLE=$O/headline/tbl_o$c.json step headline/o_2256s$c 400 python -u bench.py --steps 20 --warmup 5; done
           XOT_GEMM_TABLE=$T step headline/o_tuned2 400 python -u bench.py --steps 20 --warmup 5 ;;
    tunelog) # the tuner's isolated timings of every shuffled-weight candidate (70B and 8B at 512 sequences)
           XOT_GEMM_TUNE_LOG=1 XOT_GEMM_TABLE=$O/headline/tbl_log70.json step headline/tunelog_70b 400 python -u bench.py --steps 5 --warmup 2
           XOT_GEMM_TUNE_LOG=1 XOT_GEMM_TABLE=$O/headline/tbl_log8.json step headline/tunelog_8b 400 python -u bench.py --model llama-3-8b --batch-per-gpu 512 --steps 5 --warmup 2 ;;
    tiex)  # the cross-split tie window for the two-phase tile (XOT_GEMM_TIE_X, default 0.10) vs none, 70B and 8B
           for x in 0.10 0 0.10; do
             XOT_GEMM_TUNE_LOG=1 XOT_GEMM_TIE_X=$x XOT_GEMM_TABLE=$O/headline/tbl_x$x.json step headline/tiex_70b_$x 400 python -u bench.py --steps 20 --warmup 5
             XOT_GEMM_TUNE_LOG=1 XOT_GEMM_TIE_X=$x XOT_GEMM_TABLE=$O/headline/tbl_x${x}_8b.json step headline/tiex_8b_$x 400 python -u bench.py --model llama-3-8b --batch-per-gpu 512 --steps 20 --warmup 5; done ;;
    b384)  # 384 sequences: 192-row tiles (two-phase 1922256 offered), with the tuner's timings
           XOT_GEMM_TUNE_LOG=1 XOT_GEMM_TABLE=$O/headline/tbl384.json step headline/b384 400 python -u bench.py --batch-per-gpu 384 --steps 20 --warmup 5
           cp "$O/headline/tbl384.json" "$O/headline/tbl384_base.json"
           python - "$O/headline/tbl384_base.json" <<'PY'
import json, sys
p = sys.argv[1]; t = json.load(open(p))
for k, v in t.items():
  if isinstance(v, list) and v[0] == "big" and v[1] == 1922256: t[k] = ["big", 1920256, v[2]]
json.dump(t, open(p, "w"))
PY
           XOT_GEMM_TABLE=$O/headline/tbl384_base.json step headline/b384_base 400 python -u bench.py --batch-per-gpu 384 --steps 20 --warmup 5
           XOT_GEMM_TABLE=$O/headline/tbl384.json step headline/b384_2 400 python -u bench.py --batch-per-gpu 384 --steps 20 --warmup 5 ;;
    vtail) # decode attention skipping the unused V half of the last page (default) or not: kernel alone, then the step
           for v in 1 0 1; do XOT_ATTN_VTAIL=$v step headline/vtail_attn_$v 300 python -u tools/bench_attn_layout.py; done
           for v in 1 0 1; do XOT_ATTN_VTAIL=$v XOT_GEMM_TABLE=$O/headline/tbl_vt.json step headline/vtail_step_$v 400 python -u bench.py --steps 20 --warmup 5; done ;;
    srr)   # split-K residual RMSNorm at D = 8192: 1024 threads per row (default) vs 256
           for v in 1 0 1; do XOT_SRR_WIDE=$v XOT_GEMM_TABLE=$O/headline/tbl_srr.json step headline/srr_$v 400 python -u bench.py --steps 20 --warmup 5; done ;;
    sweep) for b in 448 512 576; do step headline/b$b 400 python -u bench.py --batch-per-gpu $b --steps 10 --warmup 3; done ;;
  esac
done

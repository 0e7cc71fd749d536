#!/bin/bash
# Round-6 headline experiments, one case per argument (each step under its own time limit, first failure ends):
#   bash tools/gpu/r6.sh bench reduce nov prof ...
# Every bench in one call shares one GEMM table (tuned once, by the first bench), so A/B arms run the same tiles.
source "$(dirname "$0")/common.sh"
T=$O/r6/gemm_table.json
mkdir -p "$O/r6"
for what in "$@"; do
  case $what in
    bench)  XOT_GEMM_TABLE=$T step r6/bench 400 python -u bench.py --steps 20 --warmup 5 ;;
    bench_a6) XOT_ATTN_DECODE=6 XOT_GEMM_TABLE=$T step r6/bench_a6 400 python -u bench.py --steps 20 --warmup 5 ;;
    bench_a3) XOT_ATTN_DECODE=3 XOT_GEMM_TABLE=$T step r6/bench_a3 400 python -u bench.py --steps 20 --warmup 5 ;;
    bench2) XOT_GEMM_TABLE=$T step r6/bench2 400 python -u bench.py --steps 20 --warmup 5 ;;
    bench_w4) cp tools/gpu/tables/decode_w4.json "$O/r6/t_w4.json" && XOT_GEMM_TABLE=$O/r6/t_w4.json step r6/bench_w4 400 python -u bench.py --steps 20 --warmup 5 ;;
    bench_w4gu) cp tools/gpu/tables/decode_w4_gateup.json "$O/r6/t_w4gu.json" && XOT_GEMM_TABLE=$O/r6/t_w4gu.json step r6/bench_w4gu 400 python -u bench.py --steps 20 --warmup 5 ;;
    reduce) step r6/reduce 120 python -u tools/bench_reduce.py ;;
    attn)   step r6/attn 200 python -u tools/bench_attn_b512.py ;;
    attn_algos) step r6/attn_algos 300 python -u tools/bench_attn_b512.py --algos 1,2,3,5,6 ;;
    attn_small) step r6/attn_small 300 python -u tools/bench_attn_small.py ;;
    b1bench) step r6/b1bench 300 python -u bench.py --model llama-3-8b --batch-per-gpu 1 --steps 64 --warmup 8 ;;
    prof)   XOT_GEMM_TABLE=$T prof r6/prof 600 python3 "$R/bench.py" --steps 6 --warmup 3
            step r6/breakdown 60 python tools/decode_breakdown.py "$(ls "$O"/r6/prof/*/*kernel_trace.csv "$O"/r6/prof/*kernel_trace.csv 2>/dev/null | head -1)" --steps 6 --json "$O/r6/breakdown.json"
            cat "$O/r6/breakdown.log" ;;
    b1)     prof r6/prof8b1 300 python3 "$R/bench.py" --model llama-3-8b --batch-per-gpu 1 --steps 16 --warmup 4
            step r6/breakdown8b1 60 python tools/decode_breakdown.py "$(ls "$O"/r6/prof8b1/*/*kernel_trace.csv "$O"/r6/prof8b1/*kernel_trace.csv 2>/dev/null | head -1)" --steps 16 --json "$O/r6/breakdown8b1.json" ;;
    ring70) # RingServer (`xot --gpus 1 --ring`) at the headline operating point: Llama-3-70B, 512 streams x 128 tokens
            step r6/ring70 1100 python -u tools/bench_serve.py --ring 1 --model llama-3-70b --concurrency 512 --max-tokens 128 --prompt-words 124 --server-log "$O/r6/ring70_server.log" ;;
    train)  step r6/train 900 python -u tools/bench_train.py --model llama-3-8b --seq 2048 --mb 2 --microbatches 4 --steps 3 --warmup 1 ;;
    tn_test) step r6/tn_test 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_train_own_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "tn or train or silu_down or relayout" ;;
    tn_test_on) XOT_DW_TN=1 step r6/tn_test_on 300 python -u -m pytest tests/test_train_own_gpu.py tests/test_pipeline_train.py -m gpu -x -q --timeout 120 --timeout-method thread ;;
    train_tn) XOT_DW_TN=1 step r6/train_tn 900 python -u tools/bench_train.py --model llama-3-8b --seq 2048 --mb 2 --microbatches 4 --steps 3 --warmup 1 ;;
    train_relayout) XOT_DW_TN=0 step r6/train_relayout 900 python -u tools/bench_train.py --model llama-3-8b --seq 2048 --mb 2 --microbatches 4 --steps 3 --warmup 1 ;;
    dw) step r6/dw 300 python -u tools/bench_dw.py ;;
    train_mb) for cfg in "4 2" "8 1" "1 8"; do set -- $cfg; step r6/train_mb$1x$2 900 python -u tools/bench_train.py --model llama-3-8b --seq 2048 --mb $1 --microbatches $2 --steps 3 --warmup 1; done ;;
    train_inline) XOT_DW_STREAM=0 step r6/train_inline 900 python -u tools/bench_train.py --model llama-3-8b --seq 2048 --mb 2 --microbatches 4 --steps 3 --warmup 1 ;;
    train_tprof) step r6/train_tprof 900 python -u tools/bench_train.py --model llama-3-8b --seq 2048 --mb 2 --microbatches 4 --steps 2 --warmup 1 --torch-prof "$O/r6/train_torch_ops.txt" ;;
    trainprof) prof r6/trainprof 900 python3 "$R/tools/bench_train.py" --mb 2 --microbatches 4 --steps 3 --warmup 1
            step r6/trainstep 60 python tools/step_window.py "$(ls "$O"/r6/trainprof/*/*kernel_trace.csv "$O"/r6/trainprof/*kernel_trace.csv 2>/dev/null | head -1)" ;;
    relayout_test) step r6/relayout_test 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k relayout ;;
    attn_train) step r6/attn_train_test 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "attention_train or deepseek" &&
                step r6/attn_train 200 python -u tools/bench_attn_train.py --reps 30 &&
                prof r6/attn_train_prof 200 python3 "$R/tools/bench_attn_train.py" --reps 10 ;;
    fnorm_test) step r6/fnorm_test 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_runner_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k "gemm_stream_norm or fused_norm or test_gemm_stream or split_equals_full or llama70b_layers" ;;
    b1_70b) step r6/b1_70b 400 python -u bench.py --batch-per-gpu 1 --steps 32 --warmup 4 ;;
    b1_70b_unfused) XOT_FUSE_NORM=0 step r6/b1_70b_unfused 400 python -u bench.py --batch-per-gpu 1 --steps 32 --warmup 4 ;;
    b1_nomerge) XOT_FUSE_MERGE=0 step r6/b1_nomerge 300 python -u bench.py --model llama-3-8b --batch-per-gpu 1 --steps 64 --warmup 8 ;;
    b1_unfused) XOT_FUSE_NORM=0 step r6/b1_unfused 300 python -u bench.py --model llama-3-8b --batch-per-gpu 1 --steps 64 --warmup 8 ;;
    b1_fused) XOT_FUSE_NORM=1 step r6/b1_fused 300 python -u bench.py --model llama-3-8b --batch-per-gpu 1 --steps 64 --warmup 8 ;;
    fnorm_diag) step r6/fnorm_diag 300 python -u tools/diag/fused_norm_diag.py ;;
    qkvattn_test) step r6/qkvattn_test 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_train_own_gpu.py tests/test_runner_gpu.py tests/test_engine_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "qkv_attention or attention_train or train or fused_grad or tied" ;;
    tests)  step r6/gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ;;
    *) echo "unknown case $what"; exit 2 ;;
  esac
done

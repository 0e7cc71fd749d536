#!/bin/bash
# The other BASELINE.json configs on one GPU: 8B and 70B batch-1 / batch-512 decode, Mixtral, model families,
# weight-only FP8, long context.   bash tools/gpu/configs.sh [dense|moe|families|fp8|long|moepp2|moepp2mx|mxdown|moepp2s|b1prof|mxprof]...  (default: dense moe)
source "$(dirname "$0")/common.sh"
for what in ${@:-dense moe}; do
  case $what in
    dense) step cfg/l8b_b1 600 python bench.py --model llama-3-8b --batch-per-gpu 1 --steps 32 --warmup 4
           step cfg/l8b_b512 600 python bench.py --model llama-3-8b --batch-per-gpu 512 --steps 16 --warmup 3
           step cfg/l70b_b1 600 python bench.py --model llama-3-70b --batch-per-gpu 1 --steps 16 --warmup 3 ;;
    moe)   step cfg/mixtral_b1 600 python bench.py --model mixtral-8x7b --batch-per-gpu 1 --steps 32 --warmup 4
           step cfg/mixtral_b512 600 python bench.py --model mixtral-8x7b --batch-per-gpu 512 --steps 8 --warmup 3 ;;
    families)
           step cfg/dsl_b256 600 python bench.py --model deepseek-coder-v2-lite --batch-per-gpu 256 --steps 16 --warmup 3
           step cfg/dsv3_8l_b256 600 python bench.py --model deepseek-v3 --layers 8 --batch-per-gpu 256 --steps 8 --warmup 3
           step cfg/phi4_b256 600 python bench.py --model phi-4-mini-instruct --batch-per-gpu 256 --steps 16 --warmup 3
           step cfg/llava_b64 600 python bench.py --model llava-1.5-7b-hf --batch-per-gpu 64 --steps 16 --warmup 3 ;;
    fp8)   for m in llama-3-70b llama-3-8b; do for b in 1 64; do
             step cfg/fp8_${m}_b$b 600 python bench.py --model $m --batch-per-gpu $b --steps 32 --warmup 4 --weight-dtype fp8
           done; done ;;
    moepp2) # 256-row expert tiles: two-phase ping-pong (default) vs base schedule
           for v in 1 0; do XOT_MOE_PP2=$v step cfg/dsl_b256_moepp2_$v 600 python bench.py --model deepseek-coder-v2-lite --batch-per-gpu 256 --steps 16 --warmup 3
             XOT_MOE_PP2=$v step cfg/dsv3_8l_b256_moepp2_$v 600 python bench.py --model deepseek-v3 --layers 8 --batch-per-gpu 256 --steps 8 --warmup 3; done ;;
    moepp2mx) # 192-row expert tiles (Mixtral): two-phase ping-pong (default) vs base schedule
           for v in 1 0 1; do XOT_MOE_PP2=$v step cfg/mixtral_b512_moepp2_$v 600 python bench.py --model mixtral-8x7b --batch-per-gpu 512 --steps 8 --warmup 3; done ;;
    mxdown) # Mixtral B=512: the grouped down GEMM's K split (default 4) and the 256-row tile
           for v in 2 8 4 6; do XOT_MOE_DN_SPLITS=$v step cfg/mixtral_b512_dn$v 600 python bench.py --model mixtral-8x7b --batch-per-gpu 512 --steps 8 --warmup 3; done
           XOT_MOE_BM=2256 step cfg/mixtral_b512_bm2256 600 python bench.py --model mixtral-8x7b --batch-per-gpu 512 --steps 8 --warmup 3 ;;
    moepp2s) # Mixtral at 128 / 256 sequences: the tuned expert tiles vs all on the two-phase 128-row tile (2128)
           for b in 256 128; do step cfg/mixtral_b${b}_tuned 600 python bench.py --model mixtral-8x7b --batch-per-gpu $b --steps 16 --warmup 3
             XOT_MOE_BM=2128 step cfg/mixtral_b${b}_2128 600 python bench.py --model mixtral-8x7b --batch-per-gpu $b --steps 16 --warmup 3; done ;;
    b1prof|mxprof) ;;
    long)  for t in 8192 32768 65536; do step long/l8b_$t 600 python -u tools/bench_long_prefill.py --model llama-3.1-8b --tokens $t; done
           step long/l70b_32768 600 python -u tools/bench_long_prefill.py --model llama-3.1-70b --tokens 32768 ;;
  esac
done
# b1prof: kernel trace of 8B batch-1 decode and its per-step breakdown
if [ "$1" = b1prof ]; then
  prof cfg/b1prof 300 python3 "$R/bench.py" --model llama-3-8b --batch-per-gpu 1 --steps 16 --warmup 4
  step cfg/b1breakdown 60 python tools/decode_breakdown.py "$(ls "$O"/cfg/b1prof/*/*kernel_trace.csv "$O"/cfg/b1prof/*kernel_trace.csv 2>/dev/null | head -1)" --steps 16 --json "$O/cfg/b1breakdown.json"
fi
# mxprof: kernel trace of Mixtral-8x7B decode at 512 sequences and its per-step breakdown
if [ "$1" = mxprof ]; then
  prof cfg/mxprof 400 python3 "$R/bench.py" --model mixtral-8x7b --batch-per-gpu 512 --steps 6 --warmup 3
  step cfg/mxbreakdown 60 python tools/decode_breakdown.py "$(ls "$O"/cfg/mxprof/*/*kernel_trace.csv "$O"/cfg/mxprof/*kernel_trace.csv 2>/dev/null | head -1)" --steps 6 --json "$O/cfg/mxbreakdown.json"
fi

#!/bin/bash
# Kernel microbenchmarks (numerics tests first).   bash tools/gpu/kernels.sh [gemm|lab|attn|prefill|moe|mla|sample]...
source "$(dirname "$0")/common.sh"
for what in ${@:-gemm attn}; do
  case $what in
    gemm)    step kern/gemm_tests 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "gemm or moe"
             step kern/gemm 600 python -u tools/bench_gemm_big.py ;;
    lab)     # standalone HIP lab (random operands, HBM-cold, variants interleaved): build it first with
             # hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/lab/gemm_lab2.hip -o tools/lab/gemm_lab2
             for a in "512 57344 8192" "2048 57344 8192" "512 8192 28672 -1 0"; do step kern/lab_${a// /_} 120 tools/lab/gemm_lab2 $a; done ;;
    attn)    step kern/attn_tests 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k attn
             step kern/attn_b512 300 python -u tools/bench_attn_b512.py
             step kern/attn_small 300 python -u tools/bench_attn_small.py ;;
    prefill) step kern/attn_prefill 300 python tools/bench_attn_prefill.py --seqs 1 --len 8192 --heads 32 --kv-heads 8 --dh 128 ;;
    moe)     step kern/moe 300 python -u tools/bench_moe.py ;;
    mla)     step kern/mla 300 python -u tools/bench_mla.py ;;
    sample)  step kern/sample 300 python -u tools/bench_sample.py ;;
  esac
done

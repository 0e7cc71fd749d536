#!/bin/bash
# Serving through the HTTP API (Llama-3-8B): streams 1 / 64 / 256, shared-prefix cache on / off, and the
# RCCL ring server rehearsed on one GPU (2 ranks over gloo).   bash tools/gpu/serve.sh [api|prefix|ring|ringload|ringload2|lanes|ring70]...
source "$(dirname "$0")/common.sh"
for what in ${@:-api}; do
  case $what in
    api)    for c in 1 64 256; do XOT_MAX_BATCH=$c step serve/c$c 400 python -u tools/bench_serve.py --model llama-3-8b --concurrency $c --max-tokens 128 --prompt-words 200; done ;;
    prefix) for pc in 1 0; do XOT_PREFIX_CACHE=$pc XOT_MAX_BATCH=64 step serve/prefix_pc$pc 400 python -u tools/bench_serve.py --model llama-3-8b --concurrency 64 --max-tokens 128 --prompt-words 400 --shared-prefix; done ;;
    ring)   step serve/ring_tests 300 python -u -m pytest tests/test_ring_serve.py tests/test_ring_health.py -x -v --timeout 200 --timeout-method thread
            XOT_DIST_BACKEND=gloo step serve/ring_run 300 python -u -m xotorch_support_jetson_amd.main run llama-3-8b --gpus 2 --prompt "Who are you?" --max-generate-tokens 24 --disable-tui ;;
    ringload)  # API load against the 2-rank ring server (gloo hand-off through host memory: a rehearsal, not RCCL speed)
            for c in 1 64; do XOT_DIST_BACKEND=gloo step serve/ring2_c$c 600 python -u tools/bench_serve.py --ring 2 --model llama-3-8b --concurrency $c --max-tokens 64 --prompt-words 16; done ;;
    ringload2)  # longer loads (round 4): 2 and 4 ranks, 64 / 256 streams x 256 tokens, and a shared-prefix workload
            for r in 2 4; do for c in 64 256; do XOT_MAX_BATCH=$c XOT_DIST_BACKEND=gloo step serve/ring${r}_c${c}_t256 600 python -u tools/bench_serve.py --ring $r --model llama-3-8b --concurrency $c --max-tokens 256 --prompt-words 16; done; done
            XOT_MAX_BATCH=64 XOT_DIST_BACKEND=gloo step serve/ring2_prefix 600 python -u tools/bench_serve.py --ring 2 --model llama-3-8b --concurrency 64 --max-tokens 128 --prompt-words 400 --shared-prefix ;;
    lanes)  # two lanes per rank vs one (rank 0 turns one lane's ids around while another lane's step is queued)
            for l in 1 2; do for c in 64 256; do XOT_RING_LANES_PER_RANK=$l XOT_MAX_BATCH=$c XOT_DIST_BACKEND=gloo step serve/ring2_c${c}_lanes$l 600 python -u tools/bench_serve.py --ring 2 --model llama-3-8b --concurrency $c --max-tokens 256 --prompt-words 16; done; done ;;
    ring70) # `xot --gpus 1` (RingServer: async lane steps) at the headline operating point: Llama-3-70B, 512 streams,
            # ~512-token prompts, 128 tokens each; compare decode_window.tok_s with bench.py
            step serve/ring1_70b_c512 1000 python -u tools/bench_serve.py --ring 1 --model llama-3-70b --concurrency 512 --max-tokens 128 --prompt-words 124 ;;
  esac
done

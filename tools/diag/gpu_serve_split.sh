#!/bin/bash
# decode-heavy serving c64 / c256 (16-word prompts, 256 tokens each), engine step split into launch / wait
mkdir -p gpurun_out
summ() { grep '"metric"' "$1" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d.get(k) for k in ('value','ms_per_step','engine_ms_per_step','engine_launch_ms_per_step','engine_wait_ms_per_step','engine_gpu_step_ms_per_step','gpu_gap_ms_mean','mean_requests_per_step','ttft_s')})"; }
for c in 64 256; do
  XOT_STEP_EVENTS=1 XOT_MAX_BATCH=$c timeout -k 10 300 python -u tools/bench_serve.py --model llama-3-8b --concurrency $c --max-tokens 256 --prompt-words 16 > gpurun_out/serve_dec_c$c.log 2>&1
  rc=$?; echo "dec c$c rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/serve_dec_c$c.log; exit $rc; }; summ gpurun_out/serve_dec_c$c.log
done

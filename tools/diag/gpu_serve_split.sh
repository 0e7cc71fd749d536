#!/bin/bash
# decode-heavy and prompt-heavy serving c64 / c256: chained engine-loop steps on (default) / off
mkdir -p gpurun_out
summ() { grep '"metric"' "$1" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d.get(k) for k in ('value','ms_per_step','engine_ms_per_step','mean_requests_per_step','ttft_s')})"; }
for ch in 1 0; do
for c in 64 256; do
  XOT_CHAIN=$ch XOT_MAX_BATCH=$c timeout -k 10 300 python -u tools/bench_serve.py --model llama-3-8b --concurrency $c --max-tokens 256 --prompt-words 16 > gpurun_out/serve_dec_chain${ch}_c$c.log 2>&1
  rc=$?; echo "chain$ch dec c$c rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/serve_dec_chain${ch}_c$c.log; exit $rc; }; summ gpurun_out/serve_dec_chain${ch}_c$c.log
done
done
for c in 64 256; do
  XOT_MAX_BATCH=$c timeout -k 10 300 python -u tools/bench_serve.py --model llama-3-8b --concurrency $c --max-tokens 128 --prompt-words 200 > gpurun_out/serve_c$c.log 2>&1
  rc=$?; echo "c$c rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/serve_c$c.log; exit $rc; }; summ gpurun_out/serve_c$c.log
done

#!/bin/bash
# serving benchmark matrix on one MI355X (Llama-3-8B): single stream, prompt-heavy c64 / c256,
# shared-prefix c64 (prefix cache on / off)
mkdir -p gpurun_out
summ() { grep '"metric"' "$1" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d.get(k) for k in ('concurrency','value','ms_per_step','mean_requests_per_step','ttft_s','prefix_cache')})"; }
for c in 1 64 256; do
  XOT_MAX_BATCH=$c timeout -k 10 400 python -u tools/bench_serve.py --model llama-3-8b --concurrency $c --max-tokens 128 --prompt-words 200 > gpurun_out/serve_c$c.log 2>&1
  rc=$?; echo "c$c rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/serve_c$c.log; exit $rc; }; summ gpurun_out/serve_c$c.log
done
for pc in 1 0; do
  XOT_PREFIX_CACHE=$pc XOT_MAX_BATCH=64 timeout -k 10 400 python -u tools/bench_serve.py --model llama-3-8b --concurrency 64 --max-tokens 128 --prompt-words 400 --shared-prefix > gpurun_out/serve_prefix_pc$pc.log 2>&1
  rc=$?; echo "prefix pc=$pc rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/serve_prefix_pc$pc.log; exit $rc; }; summ gpurun_out/serve_prefix_pc$pc.log
done

#!/bin/bash
# decode-heavy serving c64 / c256 with the engine step split into host launch / GPU wait; GIL interval A/B
mkdir -p gpurun_out
summ() { grep '"metric"' "$1" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d.get(k) for k in ('value','ms_per_step','engine_ms_per_step','engine_launch_ms_per_step','engine_wait_ms_per_step','mean_requests_per_step')})"; }
for sw in 5000 250; do
for c in 64 256; do
  XOT_SWITCH_INTERVAL_US=$sw XOT_MAX_BATCH=$c timeout -k 10 300 python -u tools/bench_serve.py --model llama-3-8b --concurrency $c --max-tokens 256 --prompt-words 16 > gpurun_out/serve_dec_sw${sw}_c$c.log 2>&1
  rc=$?; echo "sw$sw dec c$c rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/serve_dec_sw${sw}_c$c.log; exit $rc; }; summ gpurun_out/serve_dec_sw${sw}_c$c.log
done
done
timeout -k 10 300 python -u tools/diag/prof_engine_step.py 64 256 > gpurun_out/prof_engine_step.log 2>&1; echo "iso rc=$?"; grep "^B=" gpurun_out/prof_engine_step.log

#!/bin/bash
# end-to-end API serving benchmark (Node + engine + aiohttp app) on one MI355X
mkdir -p gpurun_out
for c in 1 64 256; do
  XOT_MAX_BATCH=$c timeout -k 10 500 python -u tools/bench_serve.py --model llama-3-8b --concurrency $c --max-tokens 128 --prompt-words 200 > gpurun_out/serve_c$c.log 2>&1
  rc=$?; echo "c$c rc=$rc"; grep '"metric"' gpurun_out/serve_c$c.log | cut -c1-400; [ $rc -eq 0 ] || { tail -20 gpurun_out/serve_c$c.log; exit $rc; }
done

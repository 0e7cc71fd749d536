#!/bin/bash
# serving with a shared prompt prefix: prefix-cache on vs off (Llama-3-8B, one MI355X)
mkdir -p gpurun_out
for pc in 1 0; do
  XOT_PREFIX_CACHE=$pc XOT_MAX_BATCH=64 timeout -k 10 400 python -u tools/bench_serve.py --model llama-3-8b --concurrency 64 --max-tokens 128 --prompt-words 400 --shared-prefix > gpurun_out/serve_prefix_pc$pc.log 2>&1
  rc=$?; echo "pc=$pc rc=$rc"; grep '"metric"' gpurun_out/serve_prefix_pc$pc.log | cut -c1-900; [ $rc -eq 0 ] || { tail -20 gpurun_out/serve_prefix_pc$pc.log; exit $rc; }
done

#!/bin/bash
# decode-dominated serving (short prompts, long generations) and the prompt-heavy default, c64 / c256
mkdir -p gpurun_out
for c in 64 256; do
  XOT_MAX_BATCH=$c timeout -k 10 300 python -u tools/bench_serve.py --model llama-3-8b --concurrency $c --max-tokens 256 --prompt-words 16 > gpurun_out/serve_dec_c$c.log 2>&1
  rc=$?; echo "dec c$c rc=$rc"; grep '"metric"' gpurun_out/serve_dec_c$c.log | cut -c1-700; [ $rc -eq 0 ] || { tail -20 gpurun_out/serve_dec_c$c.log; exit $rc; }
done
for c in 64 256; do
  XOT_MAX_BATCH=$c timeout -k 10 300 python -u tools/bench_serve.py --model llama-3-8b --concurrency $c --max-tokens 128 --prompt-words 200 > gpurun_out/serve_c$c.log 2>&1
  rc=$?; echo "c$c rc=$rc"; grep '"metric"' gpurun_out/serve_c$c.log | cut -c1-700; [ $rc -eq 0 ] || { tail -20 gpurun_out/serve_c$c.log; exit $rc; }
done
XOT_PROFILE=1 XOT_MAX_BATCH=64 timeout -k 10 300 python -u tools/bench_serve.py --model llama-3-8b --concurrency 64 --max-tokens 256 --prompt-words 16 > gpurun_out/serve_dec_c64_prof.log 2>&1
echo "prof rc=$?"

#!/bin/bash
# serving A/B at 64 concurrent requests: prefix cache and prefill kernel variants
mkdir -p gpurun_out/ab
for v in "XOT_PREFIX_CACHE=1 XOT_PREFILL_ATTN=2" "XOT_PREFIX_CACHE=0 XOT_PREFILL_ATTN=2" "XOT_PREFIX_CACHE=0 XOT_PREFILL_ATTN=1" "XOT_PREFIX_CACHE=1 XOT_PREFILL_ATTN=2"; do
  n=$(echo $v | tr ' =' '__')
  env $v XOT_MAX_BATCH=64 timeout -k 10 300 python -u tools/bench_serve.py --model llama-3-8b --concurrency 64 --max-tokens 128 --prompt-words 200 > gpurun_out/ab/$n.log 2>&1
  rc=$?; echo "$v rc=$rc $(grep '"metric"' gpurun_out/ab/$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ttft_s"], d["ms_per_step"], d["engine_steps"])')"; [ $rc -eq 0 ] || exit $rc
done

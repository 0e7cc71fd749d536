#!/bin/bash
# batch-1 decode (single stream) on one MI355X: Llama-3-8B and Llama-3-70B
mkdir -p gpurun_out
for m in llama-3-8b llama-3-70b; do
  timeout -k 10 400 python -u bench.py --model $m --batch-per-gpu 1 --steps 64 --warmup 8 > gpurun_out/b1_$m.log 2>&1
  rc=$?; echo "$m rc=$rc"; grep '"metric"' gpurun_out/b1_$m.log | cut -c1-260; [ $rc -eq 0 ] || exit $rc
done

#!/bin/bash
mkdir -p gpurun_out/long
for t in 8192 32768 65536; do
  timeout -k 10 600 python -u tools/bench_long_prefill.py --model llama-3.1-8b --tokens $t > gpurun_out/long/l8b_$t.log 2>&1
  rc=$?; echo "t=$t rc=$rc $(grep '^{' gpurun_out/long/l8b_$t.log)"; [ $rc -eq 0 ] || { tail -20 gpurun_out/long/l8b_$t.log; exit $rc; }
done
timeout -k 10 600 python -u tools/bench_long_prefill.py --model llama-3.1-70b --tokens 32768 > gpurun_out/long/l70b_32768.log 2>&1
rc=$?; echo "70b rc=$rc $(grep '^{' gpurun_out/long/l70b_32768.log)"; exit $rc

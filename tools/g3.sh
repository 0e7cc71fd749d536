#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/ -q -m gpu -k "attn or runner or engine or smoke" > gpurun_out/g3_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/g3_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/bench_kernels.py --attn-only --json gpurun_out/attn.json > gpurun_out/attn.log 2>&1
echo "attn rc=$?" >> gpurun_out/attn.log
timeout -k 10 600 python bench.py --steps 8 --warmup 3 > gpurun_out/bench_b512.log 2>&1
echo "bench rc=$?" >> gpurun_out/bench_b512.log

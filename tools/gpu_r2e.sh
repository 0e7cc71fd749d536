#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r2e_eng.log 2>&1
rc=$?; echo "eng rc=$rc"; tail -4 gpurun_out/r2e_eng.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2e_all.log 2>&1
rc=$?; echo "all rc=$rc"; tail -3 gpurun_out/r2e_all.log; [ $rc -eq 0 ] || exit $rc
for b in 1 64; do
  timeout -k 10 600 python bench.py --model llava-1.5-7b-hf --batch-per-gpu $b --steps 16 --warmup 3 > gpurun_out/r2e_llava_b$b.log 2>&1
  rc=$?; echo "llava b$b rc=$rc"; tail -1 gpurun_out/r2e_llava_b$b.log | cut -c1-250; [ $rc -eq 0 ] || { tail -20 gpurun_out/r2e_llava_b$b.log; exit $rc; }
done

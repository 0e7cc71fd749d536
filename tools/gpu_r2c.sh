#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -k "route_ds or mla" tests/test_runner_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2c_k.log 2>&1
rc=$?; echo "kern rc=$rc"; tail -3 gpurun_out/r2c_k.log; [ $rc -eq 0 ] || exit $rc
for mr in 24 32; do
  XOT_MOE_BIG_MIN_ROWS=$mr timeout -k 10 600 python bench.py --model deepseek-coder-v2-lite --batch-per-gpu 256 --steps 16 --warmup 3 > gpurun_out/dsl_b256_mr$mr.log 2>&1
  rc=$?; echo "mr$mr rc=$rc"; tail -1 gpurun_out/dsl_b256_mr$mr.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_dsl2 -o dsl --output-format csv -- python3 $R/bench.py --model deepseek-coder-v2-lite --batch-per-gpu 256 --steps 3 --warmup 2 > $R/gpurun_out/prof_dsl2.log 2>&1
echo "prof rc=$?"

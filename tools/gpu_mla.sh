#!/bin/bash
# MLA kernels: kernel tests, DeepSeek runner/engine tests, DeepSeek-V3 8-layer stage bench, kernel profile
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "mla" > gpurun_out/mla_tests.log 2>&1
rc=$?; tail -4 gpurun_out/mla_tests.log; [ $rc -eq 0 ] || { grep -B5 -A30 "FAIL\|Error" gpurun_out/mla_tests.log | head -60; exit $rc; }
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_runner_gpu.py tests/test_engine_gpu.py -k "deepseek" > gpurun_out/mla_tests2.log 2>&1
rc=$?; tail -4 gpurun_out/mla_tests2.log; [ $rc -eq 0 ] || exit $rc
for b in 1 256; do
  timeout -k 10 600 python bench.py --model deepseek-v3 --layers 8 --batch-per-gpu $b --steps 8 --warmup 3 > gpurun_out/mla_dsv3_8l_b$b.log 2>&1
  rc=$?; echo "dsv3 b$b rc=$rc"; tail -1 gpurun_out/mla_dsv3_8l_b$b.log | cut -c1-300; [ $rc -eq 0 ] || { tail -20 gpurun_out/mla_dsv3_8l_b$b.log; exit $rc; }
done
timeout -k 10 600 python bench.py --model deepseek-coder-v2-lite --batch-per-gpu 256 --steps 16 --warmup 3 > gpurun_out/mla_dsl_b256.log 2>&1
rc=$?; echo "dsl b256 rc=$rc"; tail -1 gpurun_out/mla_dsl_b256.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_mla -o dsv3 --output-format csv -- python3 $R/bench.py --model deepseek-v3 --layers 8 --batch-per-gpu 256 --steps 3 --warmup 2 > $R/gpurun_out/prof_mla.log 2>&1
echo "prof rc=$?"

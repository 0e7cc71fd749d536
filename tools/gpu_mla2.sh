#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/mla_pmc2
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "mla" > gpurun_out/mla_pmc2/tests.log 2>&1
rc=$?; tail -2 gpurun_out/mla_pmc2/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/bench_mla.py --batch 256 --ctx 525 > gpurun_out/mla_pmc2/bench.log 2>&1 && timeout -k 10 120 python tools/bench_mla.py --batch 64 --ctx 2048 >> gpurun_out/mla_pmc2/bench.log 2>&1
rc=$?; grep '^{' gpurun_out/mla_pmc2/bench.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace --stats -d $R/gpurun_out/mla_pmc2/p1 -o p --output-format csv -- python3 $R/tools/bench_mla.py --batch 256 --ctx 525 --iters 5 --variants 1 > $R/gpurun_out/mla_pmc2/p1.log 2>&1
echo "pmc rc=$?"

#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/prefill
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attn_prefill" > gpurun_out/prefill/tests.log 2>&1
rc=$?; tail -3 gpurun_out/prefill/tests.log; [ $rc -eq 0 ] || { grep -B2 -A25 "Error\|assert" gpurun_out/prefill/tests.log | head -60; exit $rc; }
rm -f gpurun_out/prefill/bench.log
for cfg in "--seqs 4 --len 2048 --heads 64 --kv-heads 8 --dh 128" "--seqs 1 --len 8192 --heads 32 --kv-heads 8 --dh 128" "--seqs 16 --len 512 --heads 32 --kv-heads 8 --dh 128" "--seqs 4 --len 2048 --heads 32 --kv-heads 8 --dh 64"; do
  timeout -k 10 120 python tools/bench_attn_prefill.py $cfg >> gpurun_out/prefill/bench.log 2>&1 || { tail -20 gpurun_out/prefill/bench.log; exit 1; }
done
grep '^{' gpurun_out/prefill/bench.log
cd /tmp && export TMPDIR=/tmp
i=0
for pmc in "SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" "SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS" "SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $pmc --kernel-trace -d $R/gpurun_out/prefill/p$i -o p --output-format csv -- python3 $R/tools/bench_attn_prefill.py --seqs 1 --len 8192 --heads 32 --kv-heads 8 --dh 128 --iters 3 > $R/gpurun_out/prefill/p$i.log 2>&1
  echo "pmc $i rc=$?"
done

#!/bin/bash
# MLA micro-bench + PMC counters of the wide kernel (one counter pass per run)
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/mla_pmc
timeout -k 10 120 python tools/bench_mla.py --batch 256 --ctx 525 > gpurun_out/mla_pmc/bench.log 2>&1
rc=$?; cat gpurun_out/mla_pmc/bench.log | tail -3; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/bench_mla.py --batch 64 --ctx 2048 >> gpurun_out/mla_pmc/bench.log 2>&1 && tail -2 gpurun_out/mla_pmc/bench.log || exit 1
timeout -k 10 120 python tools/bench_mla.py --batch 4 --ctx 2048 >> gpurun_out/mla_pmc/bench.log 2>&1 && tail -2 gpurun_out/mla_pmc/bench.log || exit 1
cd /tmp && export TMPDIR=/tmp
i=0
for pmc in "SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" "SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS" "SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $pmc --kernel-trace --stats -d $R/gpurun_out/mla_pmc/p$i -o p --output-format csv -- python3 $R/tools/bench_mla.py --batch 256 --ctx 525 --iters 5 --variants 1 > $R/gpurun_out/mla_pmc/p$i.log 2>&1
  echo "pmc pass $i rc=$?"
done

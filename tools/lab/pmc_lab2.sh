#!/bin/bash
# Timing + PMC passes (one counter group per run, kernel-trace only) of the lab GEMM variants on random data.
#   bash tools/lab/pmc_lab2.sh          (run on the GPU box from the repo root)
R=${GRAFT_REPO_ROOT:-$(pwd)}
L=$R/tools/lab/gemm_lab2
mkdir -p $R/gpurun_out/lab2
for args in "512 57344 8192" "2048 57344 8192" "512 8192 28672 -1 0" "512 8192 8192 -1 0"; do
  timeout -k 5 120 $L $args >> $R/gpurun_out/lab2/time.log 2>&1 || { echo "lab failed: $args rc=$?"; cat $R/gpurun_out/lab2/time.log; exit 1; }
done
cat $R/gpurun_out/lab2/time.log
cd /tmp && export TMPDIR=/tmp
i=0
for ctr in "FETCH_SIZE GRBM_GUI_ACTIVE GRBM_COUNT" \
           "TCC_HIT_sum TCC_MISS_sum TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TC_STALL_sum TD_TD_BUSY_sum" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  for v in 0 1; do
    timeout -s KILL 60 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $R/gpurun_out/lab2/p${i}v$v -o p -- $L 512 57344 8192 $v > $R/gpurun_out/lab2/p${i}v$v.log 2>&1 || { echo "pass $i v$v rc=$?"; tail -5 $R/gpurun_out/lab2/p${i}v$v.log; exit 1; }
  done
done
echo pmc done

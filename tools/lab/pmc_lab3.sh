#!/bin/bash
# PMC passes over the stream-K lab variant (4) vs the ping-pong tile (0), gate/up M=512, random operands.
R=${GRAFT_REPO_ROOT:-$(pwd)}
L=$R/tools/lab/gemm_lab2
mkdir -p $R/gpurun_out/lab3
timeout -k 5 120 $L 512 57344 8192 > $R/gpurun_out/lab3/time.log 2>&1 || { echo "lab rc=$?"; exit 1; }
cat $R/gpurun_out/lab3/time.log
cd /tmp && export TMPDIR=/tmp
i=0
for ctr in "FETCH_SIZE GRBM_GUI_ACTIVE" "TCC_HIT_sum TCC_MISS_sum TA_TA_BUSY_sum TD_TC_STALL_sum TD_TD_BUSY_sum" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES"; do
  i=$((i+1))
  for v in 4; do
    timeout -s KILL 60 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $R/gpurun_out/lab3/p${i}v$v -o p -- $L 512 57344 8192 $v > $R/gpurun_out/lab3/p${i}v$v.log 2>&1 || { echo "pass $i rc=$?"; tail -5 $R/gpurun_out/lab3/p${i}v$v.log; exit 1; }
  done
done
echo pmc done

#!/bin/bash
# PMC passes (one counter group per run, kernel-trace only) over the lab GEMM: gate/up at M=512, 256x256x64 tile.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/pmc
L=$R/tools/lab/gemm_big_lab
i=0
for ctr in "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum GRBM_GUI_ACTIVE" \
           "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TD_TC_STALL_sum TD_TD_BUSY_sum" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $R/gpurun_out/pmc/p$i -o p$i -- $L 512 57344 8192 1 $ABL 0 > $R/gpurun_out/pmc/p$i.log 2>&1 || { echo "pass $i rc=$?"; exit 1; }
done
echo done

#!/bin/bash
# PMC passes (one counter group per run, kernel-trace only) over decode attention at B=512, ctx 525.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/pmc
i=0
for ctr in "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $R/gpurun_out/pmc/a$i -o a$i -- python3 $R/tools/bench_attn_small.py --pmc ${PMC_CFG:-512,525} > $R/gpurun_out/pmc/a$i.log 2>&1 || { echo "pass $i rc=$?"; exit 1; }
done
echo done

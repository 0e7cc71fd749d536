#!/bin/bash
# rocprofv3 PMC passes over one program, one counter group per run (kernel trace only, never with sys/runtime
# traces), each pass under a hard time limit.  Groups stay within gfx950's per-block slots (8 SQ, 4 TCC with
# FETCH_SIZE = 3, 4 TCP, 2 TA, 2 TD, 2 GRBM).
#   bash tools/gpu/pmc.sh <name> <program> [args...]      e.g. bash tools/gpu/pmc.sh gateup tools/lab/gemm_lab2 512 57344 8192 0
#   (PMC_TIMEOUT=<s> per pass, default 90; summary: python tools/pmc_summary.py gpurun_out/pmc/<name>)
source "$(dirname "$0")/common.sh"
name=$1; shift
prog=$1; shift
case $prog in /*) ;; */*) prog=$R/$prog ;; *) prog=$(command -v "$prog") ;; esac  # the profiled program itself after --
i=0
for ctr in "FETCH_SIZE GRBM_GUI_ACTIVE" \
           "TCC_HIT_sum TCC_MISS_sum TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TC_STALL_sum TD_TD_BUSY_sum" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  mkdir -p "$O/pmc/$name/p$i"
  (cd /tmp && TMPDIR=/tmp timeout -s KILL ${PMC_TIMEOUT:-90} rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d "$O/pmc/$name/p$i" -o p -- "$prog" "$@" > "$O/pmc/$name/p$i.log" 2>&1)
  rc=$?; echo "pmc $name pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$O/pmc/$name/p$i.log"; exit $rc; }
done

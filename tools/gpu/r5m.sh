#!/bin/bash
# round 5: LDS / wait counters of the four-wave tile vs hipBLASLt at 4096 x 4096 x 8192
source "$(dirname "$0")/common.sh"
ctr="SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC"
ctr2="SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU"
i=0
for c in "$ctr" "$ctr2"; do
  i=$((i+1))
  for what in w4 blas; do
    mkdir -p "$O/r5m/$what$i"
    if [ $what = w4 ]; then args="--codes 4256 --no-blas"; else args="--codes none"; fi
    (cd /tmp && TMPDIR=/tmp timeout -s KILL 90 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$O/r5m/$what$i" -o p -- python3 "$R/tools/bench_gemm_w4.py" --mnk 4096,4096,8192,none $args > "$O/r5m/$what$i.log" 2>&1)
    rc=$?; echo "pmc $what $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$O/r5m/$what$i.log"; exit $rc; }
  done
done

#!/bin/bash
# Interleaved timing of the lab GEMM variants on random data (tools/lab/gemm_lab2.hip), several shapes.
R=${GRAFT_REPO_ROOT:-$(pwd)}
L=$R/tools/lab/gemm_lab2
mkdir -p $R/gpurun_out/lab
for args in "512 57344 8192" "2048 57344 8192" "512 28672 4096" "2048 28672 4096" "512 8192 28672 -1 0" "2048 8192 8192 -1 0"; do
  timeout -k 5 120 $L $args >> $R/gpurun_out/lab/time.log 2>&1 || { echo "lab failed: $args rc=$?"; cat $R/gpurun_out/lab/time.log; exit 1; }
done
cat $R/gpurun_out/lab/time.log

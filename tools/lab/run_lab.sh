#!/bin/bash
mkdir -p gpurun_out
L=tools/lab/gemm_big_lab
for args in "512 57344 8192 1 0 6" "2048 8192 8192 1 0 6" "512 8192 28672 4 0 6" "2048 57344 8192 1 0 6"; do
  timeout -k 5 90 $L $args >> gpurun_out/lab.log 2>&1 || { echo "lab failed: $args rc=$?"; cat gpurun_out/lab.log; exit 1; }
done
cat gpurun_out/lab.log

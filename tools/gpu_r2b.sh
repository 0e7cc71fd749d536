#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -k "odd_chunks or moe_layer or gemm_stream" -x -q --timeout 120 --timeout-method thread > gpurun_out/r2b_k.log 2>&1
rc=$?; echo "kern rc=$rc"; tail -3 gpurun_out/r2b_k.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ds.sh

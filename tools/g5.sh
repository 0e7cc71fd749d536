#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -k sample > gpurun_out/g5.log 2>&1 || exit $?
timeout -k 10 300 python tools/bench_sample.py >> gpurun_out/g5.log 2>&1

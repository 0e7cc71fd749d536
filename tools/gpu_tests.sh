#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/ -m gpu -q ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/gpu_tests.log 2>&1
echo "pytest rc=$?" >> gpurun_out/gpu_tests.log

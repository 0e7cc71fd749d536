#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ring_serve.py tests/test_ring_health.py -x -v --timeout 120 --timeout-method thread > gpurun_out/ring_serve_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -12 gpurun_out/ring_serve_tests.log; exit $rc

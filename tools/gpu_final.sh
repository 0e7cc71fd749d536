#!/bin/bash
# Round-end rehearsal: the driver's GPU tiers (pytest -m gpu, smoke, bench.py defaults), each under its own limit.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/final_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/final_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/final_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/final_bench.log | cut -c1-600; exit $rc

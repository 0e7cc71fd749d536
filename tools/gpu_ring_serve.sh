#!/bin/bash
# ring serving on one MI355X: the round-loop tests, then a 2-rank ring (gloo-staged, both ranks on cuda:0)
# answering one prompt through `xot run --ring --gpus 2`
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ring_serve.py tests/test_ring_health.py -x -v --timeout 120 --timeout-method thread > gpurun_out/ring_serve_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -8 gpurun_out/ring_serve_tests.log; [ $rc -eq 0 ] || exit $rc
XOT_DIST_BACKEND=gloo timeout -k 10 300 python -u -m xotorch_support_jetson_amd.main run llama-3-8b --ring --gpus 2 --prompt "Who are you?" --max-generate-tokens 24 --disable-tui > gpurun_out/ring_serve_run.log 2>&1
rc=$?; echo "ring run rc=$rc"; tail -5 gpurun_out/ring_serve_run.log; exit $rc

#!/bin/bash
# round 5: tiled prefill V write: numerics, A/B on one box (prefill time)
source "$(dirname "$0")/common.sh"
step r5v/tests 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "rope"
step r5v/on 500 python -u bench.py --steps 5 --warmup 2
XOT_ROPE_TILED=0 step r5v/off 500 python -u bench.py --steps 5 --warmup 2
grep -h "prefill" "$O"/r5v/on.log "$O"/r5v/off.log

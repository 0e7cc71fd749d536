#!/bin/bash
# round 5: full GPU suite + smoke after the attention backward v2, then the headline bench
source "$(dirname "$0")/common.sh"
step r5zf/gpu_tests 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step r5zf/smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step r5zf/headline 500 python -u bench.py --steps 20 --warmup 5

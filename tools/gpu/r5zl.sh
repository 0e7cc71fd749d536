#!/bin/bash
# round 5: headline bench (decode + the 512 x 512 prefill) with 8192- and 12288-token prefill chunks
source "$(dirname "$0")/common.sh"
step r5zl/chunk8192 500 python -u bench.py --steps 20 --warmup 5
XOT_PREFILL_CHUNK=12288 step r5zl/chunk12288 500 python -u bench.py --steps 20 --warmup 5

#!/bin/bash
# round 5: headline prefill chunk size (the tall GEMMs' M; 4096 keeps the gate/up output inside the 256 MB MALL)
source "$(dirname "$0")/common.sh"
B="python -u bench.py --steps 5 --warmup 2"
step r5t/c8192 500 $B
XOT_PREFILL_CHUNK=4096 step r5t/c4096 500 $B
XOT_PREFILL_CHUNK=16384 step r5t/c16384 500 $B
grep -h "prefill" "$O"/r5t/*.log

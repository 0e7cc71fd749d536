#!/bin/bash
# round 5: headline in-step A/B of the four-wave tile on the decode GEMMs (same tuned table, one entry forced)
source "$(dirname "$0")/common.sh"
T=$O/r5p/tbl.json
mkdir -p "$O/r5p"
XOT_GEMM_TABLE=$T step r5p/base 500 python -u bench.py --steps 20 --warmup 5
cp $T $O/r5p/tbl_base.json
python tools/gemm_table.py set $T 57344 8192 '["big", 4256, 1]' 512
XOT_GEMM_TABLE=$T step r5p/gu4256 500 python -u bench.py --steps 20 --warmup 5
python tools/gemm_table.py set $T 8192 28672 '["big", 4256, 4]' 512
XOT_GEMM_TABLE=$T step r5p/gu_dn4256 500 python -u bench.py --steps 20 --warmup 5
cp $O/r5p/tbl_base.json $T
XOT_GEMM_TABLE=$T step r5p/base2 500 python -u bench.py --steps 20 --warmup 5

#!/bin/bash
# Headline A/B: own kernels for every projection (default) vs gate/up row-major on hipBLASLt, then a kernel
# trace of the default for the per-kernel decode breakdown.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ab
mkdir -p $O
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/own.log 2>&1 || { echo "own rc=$?"; tail $O/own.log; exit 1; }
tail -1 $O/own.log | cut -c1-200
XOT_ROWMAJOR_PROJ=gu timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/gu_blas.log 2>&1 || { echo "blas rc=$?"; tail $O/gu_blas.log; exit 1; }
tail -1 $O/gu_blas.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o head --output-format csv -- python3 $R/bench.py --steps 6 --warmup 3 > $O/prof.log 2>&1 || { echo "prof rc=$?"; exit 1; }
cd $R && python tools/decode_breakdown.py $(ls $O/prof/*/*kernel_trace.csv 2>/dev/null || find $O/prof -name "*kernel_trace.csv" | head -1) --steps 6 --json $O/breakdown.json

#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run (no PMC counters here)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o bench --output-format csv -- python3 $R/bench.py --steps 4 --warmup 2 "$@" > $R/gpurun_out/prof.log 2>&1
echo "prof rc=$?" >> $R/gpurun_out/prof.log

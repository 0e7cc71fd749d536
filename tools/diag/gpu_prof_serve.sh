#!/bin/bash
# kernel trace of the decode-heavy serving bench at 256 streams (where does the GPU step time go?)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/prof_serve
XOT_BENCH_CLEAN_EXIT=1 XOT_MAX_BATCH=256 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_serve -o trace --output-format csv -- python3 $R/tools/bench_serve.py --model llama-3-8b --concurrency 256 --max-tokens 256 --prompt-words 16 > $R/gpurun_out/prof_serve.log 2>&1
echo "prof rc=$?"
grep '"metric"' $R/gpurun_out/prof_serve.log | cut -c1-300
f=$(find $R/gpurun_out/prof_serve -name "*kernel_stats.csv" | head -n1); head -25 "$f" | cut -c1-220

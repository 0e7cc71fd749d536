#!/bin/bash
# short kernel-trace profile of a training step (Llama-3-8B, seq 2048); prints the attention kernel rows
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/prof_train
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_train -o trace --output-format csv -- python3 $R/tools/bench_train.py --microbatches 4 --steps 1 --warmup 1 > $R/gpurun_out/prof_train.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find $R/gpurun_out/prof_train -name '*kernel_stats.csv' | head -1); grep attn_train "$f" | sed 's/(.*)"/"/' | cut -d, -f1-5

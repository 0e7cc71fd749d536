#!/bin/bash
# kernel-trace profile of a short training run (Llama-3-8B, seq 2048)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/prof_train
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_train -o trace --output-format csv -- python3 $R/tools/bench_train.py --steps 3 --warmup 1 > $R/gpurun_out/prof_train.log 2>&1
echo "prof rc=$?"

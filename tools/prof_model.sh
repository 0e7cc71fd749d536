#!/bin/bash
# kernel-trace profile of a short bench run of one model / batch: MODEL=... B=... bash tools/prof_model.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/prof_$TAG
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o trace --output-format csv -- python3 $R/bench.py --model $MODEL --batch-per-gpu $B --steps 3 --warmup 2 > $R/gpurun_out/prof_$TAG.log 2>&1
echo "prof rc=$?"

#!/bin/bash
# rocprofv3 kernel stats of the headline bench (Llama-3-70B, 512 sequences, one GPU)
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/prof_head
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_head -o head --output-format csv -- python3 $R/bench.py --steps 8 --warmup 3 > $R/gpurun_out/prof_head/bench.log 2>&1
echo "prof rc=$?"; tail -1 $R/gpurun_out/prof_head/bench.log | cut -c1-300

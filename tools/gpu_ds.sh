#!/bin/bash
# DeepSeek-Coder-V2-Lite (MLA + DeepSeekMoE, full 27 layers) and Phi-4-mini decode on one MI355X, + kernel profile
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
run() {
  local name=$1; shift
  timeout -k 10 600 python $R/bench.py "$@" > $R/gpurun_out/cfg_$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; tail -1 $R/gpurun_out/cfg_$name.log | cut -c1-300
  if [ $rc -ne 0 ]; then tail -20 $R/gpurun_out/cfg_$name.log; exit $rc; fi
}
run dsl_b1 --model deepseek-coder-v2-lite --batch-per-gpu 1 --steps 32 --warmup 4
run dsl_b256 --model deepseek-coder-v2-lite --batch-per-gpu 256 --steps 16 --warmup 3
run phi4_b1 --model phi-4-mini-instruct --batch-per-gpu 1 --steps 32 --warmup 4
run phi4_b256 --model phi-4-mini-instruct --batch-per-gpu 256 --steps 16 --warmup 3
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_dsl -o dsl --output-format csv -- python3 $R/bench.py --model deepseek-coder-v2-lite --batch-per-gpu 256 --steps 3 --warmup 2 > $R/gpurun_out/prof_dsl.log 2>&1
echo "prof rc=$?"

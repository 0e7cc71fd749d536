#!/bin/bash
# GPU tests, headline bench, then a kernel-trace profile of a short bench run.
mkdir -p gpurun_out
run() {  # run <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/steps.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -20 gpurun_out/$name.log; exit $rc; fi
}
run gpu_tests 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread
run bench 900 python -u bench.py
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o bench --output-format csv -- python3 $R/bench.py --steps 3 --warmup 2 > $R/gpurun_out/prof.log 2>&1
echo "prof rc=$?" | tee -a $R/gpurun_out/steps.log

#!/bin/bash
# GPU round script: every GPU step has its own time limit; stop at the first fault/abort/timeout.
mkdir -p gpurun_out
run() {  # run <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
run t2 300 python -m pytest tests/test_kernels_gpu.py tests/test_runner_gpu.py -x -q
run bench_small 300 python bench.py --steps 5 --warmup 2 --layers 8 --batch-per-gpu 64
run bench_full 600 python bench.py --steps 10 --warmup 3

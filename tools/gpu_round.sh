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
run t2 600 python -m pytest tests/ -m gpu -q
run bench_b128 600 python bench.py --steps 10 --warmup 3 --batch-per-gpu 128
run bench_b256 600 python bench.py --steps 10 --warmup 3 --batch-per-gpu 256

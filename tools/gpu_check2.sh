#!/bin/bash
# kernel tests, GEMM policy bench, then the headline bench
mkdir -p gpurun_out
run() {  # run <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/steps.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
run gpu_tests 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread
run gemm 600 python -u tools/bench_gemm_big.py --ms 256,512,8192 --json gpurun_out/bench_gemm_big.json
run bench 900 python -u bench.py

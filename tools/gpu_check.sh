#!/bin/bash
# Full GPU check of the tree: GPU tests, smoke, default bench.  Each step has its own time limit;
# the script stops at the first fault / abort / timeout (no retries).
mkdir -p gpurun_out
run() {  # run <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
run gpu_tests 900 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"}
run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
[ -n "$NO_BENCH" ] || run bench 900 python -u bench.py ${BENCH_ARGS}

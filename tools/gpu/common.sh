# Shared helpers of the GPU scripts (sourced).  Every GPU step runs under its own time limit; the first
# failure ends the script (never retried).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "${BASH_SOURCE[0]}")/../.." && pwd)}
cd "$R"
O=$R/gpurun_out
mkdir -p "$O"
step() {  # step <name> <seconds> <command...>: log to gpurun_out/<name>.log, stop on failure
  local name=$1 secs=$2; shift 2
  mkdir -p "$(dirname "$O/$name.log")"
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -h '^{' "$O/$name.log" | tail -1 | cut -c1-220)"
  [ $rc -eq 0 ] || { tail -25 "$O/$name.log"; exit $rc; }
}
prof() {  # prof <name> <seconds> <program args...>: rocprofv3 kernel trace + stats (program right after --)
  local name=$1 secs=$2; shift 2
  mkdir -p "$O/$name"
  (cd /tmp && TMPDIR=/tmp timeout -k 10 "$secs" rocprofv3 --kernel-trace --stats -d "$O/$name" -o trace \
     --output-format csv -- "$@" > "$O/$name.log" 2>&1)
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -25 "$O/$name.log"; exit $rc; }
}

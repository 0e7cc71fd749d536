#!/bin/bash
# Power / clock samples (rocm-smi, read-only) around one GPU command: bash tools/gpu/power.sh <name> <secs> <cmd...>
source "$(dirname "$0")/common.sh"
name=$1; secs=$2; shift 2
mkdir -p "$O/power"
( while true; do echo "t=$(date +%s.%N)"; rocm-smi --showpower --showclocks --showuse 2>/dev/null | grep -E "Power|sclk|fclk|mclk|GPU use" ; sleep 0.25; done ) > "$O/power/$name.smi" 2>&1 &
mon=$!
timeout -k 10 "$secs" "$@" > "$O/power/$name.log" 2>&1
rc=$?
kill $mon 2>/dev/null; wait $mon 2>/dev/null
echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -20 "$O/power/$name.log"; exit $rc; }

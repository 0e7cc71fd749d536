#!/bin/bash
# round 5: four-wave tile lab: per-stage interval probes (s_memtime) and schedule variants
source "$(dirname "$0")/common.sh"
mkdir -p "$O/r5f"
run() { timeout -k 5 60 tools/lab/w4_$1 $2 $3 $4 20 ${5:-4} >> "$O/r5f/lab7.log" 2>&1 || { echo "lab $* rc=$?"; tail -5 "$O/r5f/lab7.log"; exit 1; }; }
for v in base nb1 nvm nb2 nvmb2 nall base; do
  for s in "4096 4096 8192" "4096 28672 4096"; do run $v $s; done
done
cat "$O/r5f/lab7.log"

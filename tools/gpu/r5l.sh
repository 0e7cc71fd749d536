#!/bin/bash
# round 5: fresh decode breakdowns -- the headline (70B, 512 sequences) and 8B batch 1
source "$(dirname "$0")/common.sh"
prof r5l/prof70 600 python3 "$R/bench.py" --steps 6 --warmup 3
step r5l/breakdown70 60 python tools/decode_breakdown.py "$(ls "$O"/r5l/prof70/*kernel_trace.csv | head -1)" --steps 6 --json "$O/r5l/breakdown70.json"
prof r5l/prof8b1 300 python3 "$R/bench.py" --model llama-3-8b --batch-per-gpu 1 --steps 16 --warmup 4
step r5l/breakdown8b1 60 python tools/decode_breakdown.py "$(ls "$O"/r5l/prof8b1/*kernel_trace.csv | head -1)" --steps 16 --json "$O/r5l/breakdown8b1.json"

#!/bin/bash
# round 5: batch-1 decode with the in-launch merges (split-K combine, attention partition merge) vs the merge kernels
source "$(dirname "$0")/common.sh"
B1="python -u bench.py --model llama-3-8b --batch-per-gpu 1 --steps 64 --warmup 8 --prompt-len 512"
step r5zi/b1_base 300 $B1
XOT_SPLITK_IN_LAUNCH=1 step r5zi/b1_splitk 300 $B1
XOT_ATTN_TICKETS=1 step r5zi/b1_tickets 300 $B1
XOT_SPLITK_IN_LAUNCH=1 XOT_ATTN_TICKETS=1 step r5zi/b1_both 300 $B1
step r5zi/b1_base2 300 $B1

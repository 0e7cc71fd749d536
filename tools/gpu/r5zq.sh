#!/bin/bash
# round 5: PMC of the training attention backward kernels, v2 vs v1 (MFMA busy, LDS instructions / bank conflicts)
source "$(dirname "$0")/common.sh"
bash "$R/tools/gpu/pmc.sh" attn_bwd_v2 python3 "$R/tools/bench_attn_train.py" --reps 3 && \
XOT_TRAIN_DQ_V1=1 XOT_TRAIN_DKDV_V1=1 bash "$R/tools/gpu/pmc.sh" attn_bwd_v1 python3 "$R/tools/bench_attn_train.py" --reps 3 && \
python tools/pmc_summary.py "$O/pmc/attn_bwd_v2" > "$O/pmc/attn_bwd_v2.txt" && \
python tools/pmc_summary.py "$O/pmc/attn_bwd_v1" > "$O/pmc/attn_bwd_v1.txt"

#!/bin/bash
# round 5: training attention kernels in isolation (v2 dQ / dK-dV vs v1)
source "$(dirname "$0")/common.sh"
step r5zd/attn_v2 120 python -u tools/bench_attn_train.py
XOT_TRAIN_DQ_V1=1 step r5zd/attn_dq1 120 python -u tools/bench_attn_train.py
XOT_TRAIN_DQ_V1=1 XOT_TRAIN_DKDV_V1=1 step r5zd/attn_v1 120 python -u tools/bench_attn_train.py
step r5zd/attn_v2b 120 python -u tools/bench_attn_train.py

#!/bin/bash
# Multi-GPU headline diagnostics that fit ONE MI355X (the driver runs the real 2/4/8-GPU bench):
#   stage8 / stage4 / stage2   one pp-N ring stage at 512 sequences (tools/bench_stage.py): the per-tick time of
#                              first / middle / last stages -> the predicted node tok/s
#   rehearse8                  the exact bench.py torchrun command, 8 ranks sharing this GPU over gloo (host-staged
#                              hand-off; real kernels, HIP graphs, split head), with per-rank stage / recv-wait stats
#   bash tools/gpu/scale.sh [stage8|stage4|stage2|rehearse8]...
source "$(dirname "$0")/common.sh"
mkdir -p "$O/scale"
for what in ${@:-stage8 rehearse8}; do
  case $what in
    stage8) step scale/stage8 600 python -u tools/bench_stage.py --world 8 --ranks 0,3,7 --json "$O/scale/stage8.json" ;;
    stage4) step scale/stage4 600 python -u tools/bench_stage.py --world 4 --ranks 0,3 --json "$O/scale/stage4.json" ;;
    stage2) step scale/stage2 600 python -u tools/bench_stage.py --world 2 --ranks 0,1 --json "$O/scale/stage2.json" ;;
    rehearse8) XOT_DIST_BACKEND=gloo step scale/rehearse8 900 python -m torch.distributed.run --nnodes=1 \
                 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 8 --batch-per-gpu 32 \
                 --steps 6 --warmup 2 ;;
  esac
done

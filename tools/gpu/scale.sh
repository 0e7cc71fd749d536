#!/bin/bash
# Multi-GPU headline diagnostics that fit ONE MI355X (the driver runs the real 2/4/8-GPU bench):
#   stage8 / stage4 / stage2   one pp-N ring stage at 512 sequences (tools/bench_stage.py): the per-tick time of
#                              first / middle / last stages -> the predicted node tok/s
#   rehearse8                  the exact bench.py torchrun command, 8 ranks sharing this GPU over gloo (host-staged
#                              hand-off; real kernels, HIP graphs, split head), with per-rank stage / recv-wait stats
#   mixstage8                  the same stage timing for Mixtral-8x7B (BASELINE config 4)
#   trainstage8                one pp8 stage of the Llama-3-8B fine-tune (BASELINE config 5): 4 layers + embedding
#                              + LM head / CE on one GPU, 8 micro-batches of 2 x 2048 tokens (an upper bound on a stage)
#   trainrehearse8             the pp8 training command, 8 gloo ranks sharing this GPU (real kernels, 1F1B)
#   bash tools/gpu/scale.sh [stage8|stage4|stage2|rehearse8|mixstage8|trainstage8|trainrehearse8]...
source "$(dirname "$0")/common.sh"
mkdir -p "$O/scale"
for what in ${@:-stage8 rehearse8}; do
  case $what in
    stage8) step scale/stage8 600 python -u tools/bench_stage.py --world 8 --ranks 0,3,7 --json "$O/scale/stage8.json" ;;
    headsplit) for f in 0.6 0.7; do XOT_HEAD_SPLIT=$f step scale/headsplit_$f 600 python -u tools/bench_stage.py --world 8 \
                 --ranks 0,7 --json "$O/scale/headsplit_$f.json"; done ;;
    stage4) step scale/stage4 600 python -u tools/bench_stage.py --world 4 --ranks 0,3 --json "$O/scale/stage4.json" ;;
    stage2) step scale/stage2 600 python -u tools/bench_stage.py --world 2 --ranks 0,1 --json "$O/scale/stage2.json" ;;
    mixstage8) step scale/mixstage8 600 python -u tools/bench_stage.py --model mixtral-8x7b --world 8 --ranks 0,3,7 \
                 --json "$O/scale/mixstage8.json" ;;
    trainstage8) step scale/trainstage8 600 python -u tools/bench_train.py --model llama-3-8b --layers 4 --mb 2 \
                 --microbatches 8 --steps 3 --warmup 1 --schedule 1f1b ;;
    trainrehearse8) XOT_DIST_BACKEND=gloo step scale/trainrehearse8 900 python -m torch.distributed.run --nnodes=1 \
                 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29562 tools/bench_train.py --gpus 8 \
                 --model llama-3-8b --mb 1 --microbatches 8 --steps 2 --warmup 1 --schedule 1f1b ;;
    rehearse8) XOT_DIST_BACKEND=gloo step scale/rehearse8 900 python -m torch.distributed.run --nnodes=1 \
                 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 8 --batch-per-gpu 32 \
                 --steps 6 --warmup 2 ;;
  esac
done

#!/bin/bash
# 2-rank ring rehearsal of bench.py on one MI355X (gloo-staged hand-off, both ranks on cuda:0)
mkdir -p gpurun_out
XOT_DIST_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29633 bench.py --gpus 2 --model llama-3-8b --batch-per-gpu 128 --steps 6 --warmup 2 > gpurun_out/bench_2rank.log 2>&1
rc=$?; echo "rc=$rc"; grep '"metric"' gpurun_out/bench_2rank.log | cut -c1-400; [ $rc -eq 0 ] || tail -20 gpurun_out/bench_2rank.log; exit $rc

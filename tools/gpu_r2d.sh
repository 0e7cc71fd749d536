#!/bin/bash
# 2-rank ring rehearsal over gloo on one GPU (logic of the N>1 bench path), DeepSeek-V3 stage-sized decode
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
XOT_DIST_BACKEND=gloo timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 4 --warmup 2 --batch-per-gpu 64 > gpurun_out/r2d_gloo2.log 2>&1
rc=$?; echo "gloo2 rc=$rc"; grep '"metric"' gpurun_out/r2d_gloo2.log | cut -c1-300; [ $rc -eq 0 ] || { tail -30 gpurun_out/r2d_gloo2.log; exit $rc; }
for b in 1 256; do
  timeout -k 10 600 python bench.py --model deepseek-v3 --layers 8 --batch-per-gpu $b --steps 8 --warmup 3 > gpurun_out/r2d_dsv3_8l_b$b.log 2>&1
  rc=$?; echo "dsv3 b$b rc=$rc"; tail -1 gpurun_out/r2d_dsv3_8l_b$b.log | cut -c1-300; [ $rc -eq 0 ] || { tail -20 gpurun_out/r2d_dsv3_8l_b$b.log; exit $rc; }
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_dsv3 -o dsv3 --output-format csv -- python3 $R/bench.py --model deepseek-v3 --layers 8 --batch-per-gpu 256 --steps 3 --warmup 2 > $R/gpurun_out/prof_dsv3.log 2>&1
echo "prof rc=$?"

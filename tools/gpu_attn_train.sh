#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "attention_train" > gpurun_out/attn_train_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/attn_train_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/bench_train.py --model llama-3-8b --seq 2048 --mb 1 --microbatches 8 --steps 3 --warmup 1 > gpurun_out/train_8b.log 2>&1
rc=$?; echo "train rc=$rc"; tail -2 gpurun_out/train_8b.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_train -o run -- python3 tools/bench_train.py --model llama-3-8b --seq 2048 --mb 1 --microbatches 4 --steps 1 --warmup 1 > gpurun_out/prof_train.log 2>&1
echo "prof rc=$?"
f=$(find gpurun_out/prof_train -name '*kernel_stats.csv' | head -1); grep attn_train "$f" | cut -d, -f1-5 | sed 's/(.*)"/"/'

#!/bin/bash
# round 5, first GPU pass: the new / changed GPU tests, training GEMM table at T=4096, train bench + profile
source "$(dirname "$0")/common.sh"
step r5a/tests 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_train_own_gpu.py \
  tests/test_runner_gpu.py::test_decode_tick_issues_no_host_sync tests/test_runner_gpu.py::test_fused_head_ce_matches_logits_path \
  tests/test_runner_gpu.py::test_moe_training_gpu tests/test_engine_gpu.py::test_training_gpu_matches_cpu \
  tests/test_ring_serve.py::test_ring_server_tokens_equal_ring_stage_gpu tests/test_ring_serve.py::test_ring_server_on_gpu tests/test_kernels_gpu.py -k "gemm_sk or vision_tower or train or ragged or no_host_sync or fused_head or moe_training or ring_server"
step r5a/train_gemms 300 python -u tools/bench_train_gemms.py --tokens 4096
step r5a/train 600 python -u tools/bench_train.py --model llama-3-8b --seq 2048 --mb 2 --microbatches 4 --steps 3 --warmup 1
prof r5a/trainprof 600 python3 "$R/tools/bench_train.py" --mb 2 --microbatches 4 --steps 2 --warmup 1

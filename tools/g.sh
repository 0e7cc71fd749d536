mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -k "gemm_stream" > gpurun_out/ts.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/ts.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python tools/bench_kernels.py --gemm-only --json gpurun_out/bench_gemm.json > gpurun_out/bg.log 2>&1; echo "bench rc=$?" >> gpurun_out/bg.log

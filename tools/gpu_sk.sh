set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/bench_gemm_sk.py --ms 512,2048 --ops gate_up,down,qkv,o,gate_up_8b --json gpurun_out/r3_gemm_sk.json > gpurun_out/r3_gemm_sk.log 2>&1 || { echo "sk bench rc=$?"; tail -30 gpurun_out/r3_gemm_sk.log; exit 1; }
cat gpurun_out/r3_gemm_sk.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r3_bench_base.log 2>&1; echo "bench rc=$?"; tail -3 gpurun_out/r3_bench_base.log

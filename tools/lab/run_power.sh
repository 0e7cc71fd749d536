set -o pipefail
# long single-variant loops (LAB_ROUNDS x 10 calls) with rocm-smi power / clock sampling
export LAB_ROUNDS=1500
bash tools/gpu/power.sh gu512 120 tools/lab/gemm_lab3 512 57344 8192 1 0 && \
bash tools/gpu/power.sh gu2048 160 tools/lab/gemm_lab3 2048 57344 8192 1 0 && \
LAB_ROUNDS=3000 bash tools/gpu/power.sh down512 120 tools/lab/gemm_lab3 512 8192 28672 4 0

set -o pipefail
L=tools/lab/gemm_lab3
mkdir -p gpurun_out/lab3
for a in "512 57344 8192 1" "512 8192 28672 4" "512 10240 8192 3" "512 8192 8192 2" "448 57344 8192 1"; do
  timeout -k 5 120 $L $a >> gpurun_out/lab3/time.log 2>&1 || { echo "lab failed: $a rc=$?"; tail -20 gpurun_out/lab3/time.log; exit 1; }
done
cat gpurun_out/lab3/time.log

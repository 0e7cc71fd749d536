set -o pipefail
L=tools/lab/gemm_lab2
mkdir -p gpurun_out/lab4
for a in "512 57344 8192" "2048 57344 8192" "2048 28672 4096" "512 8192 28672 -1 0"; do
  timeout -k 5 120 $L $a >> gpurun_out/lab4/time.log 2>&1 || { echo "lab failed: $a rc=$?"; tail -20 gpurun_out/lab4/time.log; exit 1; }
done
cat gpurun_out/lab4/time.log

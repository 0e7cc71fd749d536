set -o pipefail
L=tools/lab/gemm_lab4
mkdir -p gpurun_out/lab4
for a in "512 57344 8192 1" "2048 57344 8192 1" "512 8192 28672 4"; do
  timeout -k 5 150 $L $a >> gpurun_out/lab4/time.log 2>&1 || { echo "lab failed: $a rc=$?"; tail -20 gpurun_out/lab4/time.log; exit 1; }
done
cat gpurun_out/lab4/time.log
LAB_ROUNDS=1500 bash tools/gpu/power.sh pp_512 120 $L 512 57344 8192 1 0 && LAB_ROUNDS=1500 bash tools/gpu/power.sh ppagpr_512 120 $L 512 57344 8192 1 1

#!/bin/bash
# kernel-trace breakdown of Llama-3-8B decode at B=64 and B=256 (the serving batch sizes)
R=${GRAFT_REPO_ROOT:-$(pwd)}
for B in 64 256; do
  MODEL=llama-3-8b B=$B TAG=8b_b$B bash $R/tools/prof_model.sh || exit 1
  cd $R && python3 tools/decode_breakdown.py "$(ls gpurun_out/prof_8b_b$B/*/*kernel_trace.csv gpurun_out/prof_8b_b$B/*kernel_trace.csv 2>/dev/null | head -n1)" --steps 3 --json gpurun_out/decode_breakdown_8b_b$B.json > gpurun_out/decode_breakdown_8b_b$B.txt 2>&1; echo "bd rc=$?"; head -20 gpurun_out/decode_breakdown_8b_b$B.txt
done

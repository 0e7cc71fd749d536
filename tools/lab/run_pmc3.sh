set -o pipefail
# PMC passes of the gate/up M = 512 tile shapes: 256 x 256 ping-pong (variant 0) vs 512 x 128 nt (variant 2),
# plus power / clock under long loops of each
export LAB_ROUNDS=3
bash tools/gpu/pmc.sh gu512_pp tools/lab/gemm_lab3 512 57344 8192 1 0 && \
bash tools/gpu/pmc.sh gu512_512x128 tools/lab/gemm_lab3 512 57344 8192 1 2 && \
python tools/pmc_summary.py gpurun_out/pmc/gu512_pp --match gemm_big --last 20 && \
python tools/pmc_summary.py gpurun_out/pmc/gu512_512x128 --match gemm_big --last 20 && \
LAB_ROUNDS=1500 bash tools/gpu/power.sh gu512_512x128 120 tools/lab/gemm_lab3 512 57344 8192 1 2

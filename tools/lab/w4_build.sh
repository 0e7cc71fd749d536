#!/bin/bash
# build the four-wave tile's lab variants (CPU side): tools/lab/w4_<name>
set -e
cd "$(dirname "$0")"
C=../../xotorch_support_jetson_amd/csrc
b() { local name=$1; shift; /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -DVARIANT="\"$name\"" "$@" -I$C w4_lab.hip -o w4_$name & }
b base
b probe -DW4_PROBE=1
b probe_abl1 -DW4_PROBE=1 -DW4_ABL=1
b probe_abl4 -DW4_PROBE=1 -DW4_ABL=4
b probe_abl7 -DW4_PROBE=1 -DW4_ABL=7
b s24_32 -DW4_B1=24 -DW4_B2=32
b s20_24 -DW4_B1=20 -DW4_B2=24
wait
ls -la w4_*

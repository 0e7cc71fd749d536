#!/bin/bash
# build the four-wave tile's lab variants (CPU side): tools/lab/w4_<name>
set -e
cd "$(dirname "$0")"
C=../../xotorch_support_jetson_amd/csrc
b() { local name=$1; shift; /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -DVARIANT="\"$name\"" "$@" -I$C w4_lab.hip -o w4_$name & }
b base
b r2a -DW4_RSP=2 -DW4_B1=40 -DW4_B2=16
b r2b -DW4_RSP=2 -DW4_B1=32 -DW4_B2=24
b r2c -DW4_RSP=2 -DW4_B1=36 -DW4_B2=20
b nonop -DW4_ABL=8
b s24_32 -DW4_B1=24 -DW4_B2=32
b probe_abl6 -DW4_PROBE=1 -DW4_ABL=6
wait
ls -la w4_*

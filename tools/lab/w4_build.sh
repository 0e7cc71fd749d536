#!/bin/bash
# build the four-wave tile's lab variants (CPU side): tools/lab/w4_<name>
set -e
cd "$(dirname "$0")"
C=../../xotorch_support_jetson_amd/csrc
b() { local name=$1; shift; /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -DVARIANT="\"$name\"" "$@" -I$C w4_lab.hip -o w4_$name & }
b base
b cvis -DW4_ASMRD=0
b nonop -DW4_ABL=8
wait
ls -la w4_*

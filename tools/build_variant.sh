#!/bin/bash
# A library build with extra compile definitions into its own directory (for same-box A/B runs: PRT_LIB_DIR=<dir>,
# tools/ab3.sh). usage: tools/build_variant.sh <dir> "<-DNAME=VALUE ...>"   (the in-tree librt_host.so is copied along)
cd "$(dirname "$0")/.." || exit 1
dir=$1; defs=$2
mkdir -p "$dir"
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -fno-slp-vectorize $defs \
    -fhip-fp32-correctly-rounded-divide-sqrt -fPIC -Wall -Iinclude -Iparallel-ray-tracer_amd/csrc -shared \
    -o "$dir/librt_hip.so" parallel-ray-tracer_amd/csrc/hip/rt_hip.hip -Lparallel-ray-tracer_amd/lib -lrt_host -ldl \
    -Wl,-rpath,'$ORIGIN' || exit 1
cp parallel-ray-tracer_amd/lib/librt_host.so "$dir/"

#!/usr/bin/env bash
# Build librvcp.so with extra kernel -D flags into tools/build/var_<name>/ (experiments only;
# select it at run time with RVCP_LIB=...).  Usage: tools/build_variant.sh NAME -DFOO=1 ...
set -eu
cd "$(dirname "$0")/../rvcp-real-time-path-tracer_amd/csrc"
make -s
name=$1; shift
out=../../tools/build/var_$name
mkdir -p "$out"
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -fno-fast-math -fno-slp-vectorize -Wno-unused-function"
/opt/rocm/bin/hipcc $FLAGS "$@" -c -o "$out/rvcp_kernels.o" rvcp_kernels.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$out/librvcp.so" "$out/rvcp_kernels.o" \
    build/rvcp_mandelbrot.o build/rvcp_host.o build/rvcp_bvh.o build/rvcp_scene_prep.o build/rvcp_jit.o -ldl
echo "$out/librvcp.so"

#!/usr/bin/env bash
# Build librvcp.so with extra -D flags (every object, so host and kernels agree) into
# tools/build/var_<name>/ (experiments only; select it at run time with RVCP_LIB=...).
#   tools/build_variant.sh NAME -DFOO=1 ...
set -eu
cd "$(dirname "$0")/../rvcp-real-time-path-tracer_amd/csrc"
make -s build/rvcp_jit_src.h
name=$1; shift
out=../../tools/build/var_$name
mkdir -p "$out"
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -fno-fast-math -fno-slp-vectorize -Wno-unused-function"
for src in rvcp_kernels.hip rvcp_mandelbrot.hip; do
  /opt/rocm/bin/hipcc $FLAGS "$@" -c -o "$out/${src%.*}.o" $src &
done
for src in rvcp_host.cpp rvcp_bvh.cpp rvcp_scene_prep.cpp rvcp_jit.cpp; do
  /opt/rocm/bin/hipcc $FLAGS "$@" -x hip -c -o "$out/${src%.*}.o" $src &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$out/librvcp.so" "$out"/*.o -ldl
echo "$out/librvcp.so"

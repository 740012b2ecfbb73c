#!/usr/bin/env bash
# Same-box A/B of LLVM scheduler options for the hipRTC-compiled specialised kernels
# (RVCP_JIT_FLAGS, comma-separated), C3 and C2 frames, via tools/env_ab.sh.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
# environment knobs exist only in the debug build of the library (csrc: make debug)
export RVCP_LIB=${RVCP_LIB:-rvcp-real-time-path-tracer_amd/csrc/build/librvcp_debug.so}
for s in "RVCP_JIT_FLAGS=-mllvm,-amdgpu-sched-strategy=max-ilp" "RVCP_JIT_FLAGS=-mllvm,-amdgpu-schedule-metric-bias=0" "RVCP_JIT_FLAGS=-mllvm,-amdgpu-sched-strategy=iterative-ilp"; do
  timeout -k 10 300 bash tools/env_ab.sh "$s" "" "--size 384 --spp 10"
done

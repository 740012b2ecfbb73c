#!/usr/bin/env bash
# Same-box A/B of the mode-2 kernel's occupancy (RVCP_LEGACY_MIN_WAVES through RVCP_JIT_FLAGS
# for the hipRTC-specialised mode-2 kernel): C3 frame in mode 2 and the sphere room.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
# environment knobs exist only in the debug build of the library (csrc: make debug)
export RVCP_LIB=${RVCP_LIB:-rvcp-real-time-path-tracer_amd/csrc/build/librvcp_debug.so}
for w in 6 7; do
  timeout -k 10 300 bash tools/env_ab.sh "RVCP_JIT_FLAGS=-DRVCP_LEGACY_MIN_WAVES=$w" \
      "--integrator 1 --spp 30" "--integrator 1 --scene spheres --spp 5"
done

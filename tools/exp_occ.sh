#!/usr/bin/env bash
# Occupancy / tail experiment: variant 3 C3 frames under different residency limits.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for cfg in "default::" "cap3:RVCP_DEBUG_BLOCKS_PER_CU=3:" "cap2:RVCP_DEBUG_BLOCKS_PER_CU=2:" "w5::rvcp-real-time-path-tracer_amd/csrc/build/variants/librvcp_w5.so"; do
  name=${cfg%%:*}; rest=${cfg#*:}; envv=${rest%%:*}; lib=${rest#*:}
  echo "== $name"
  env $envv RVCP_LIB=$lib timeout -k 10 120 python tools/frames.py --variant 3 --frames 4 || exit $?
done

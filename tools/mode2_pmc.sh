#!/usr/bin/env bash
# SQ / GRBM counters of the mode-2 kernel (sphere room 1024^2 SPP=5, 5 frames); one pass.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE -d gpurun_out/mode2_pmc -o run --output-format csv -- python3 tools/frames.py --integrator 1 --scene spheres --frames 5 --spp 5 > gpurun_out/mode2_pmc.log 2>&1
rc=$?
tail -3 gpurun_out/mode2_pmc.log
exit $rc

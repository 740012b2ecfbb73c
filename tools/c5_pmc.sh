#!/usr/bin/env bash
# PMC passes on the C5 bench (one frame): HBM traffic (FETCH_SIZE, WRITE_SIZE) and VALU
# utilisation (SQ_INSTS_VALU, GRBM_GUI_ACTIVE), each counter set in its own rocprofv3 run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
B="python3 bench.py --workload c5 --steps 1 --warmup 0 --no-cpu-baseline"
for p in "FETCH_SIZE:c5f" "WRITE_SIZE:c5w" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES:c5sq" "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES:c5g"; do
  ctr=${p%%:*}; name=${p##*:}
  timeout -k 10 400 rocprofv3 --pmc $ctr -d gpurun_out/$name -o run --output-format csv -- $B > gpurun_out/$name.log 2>&1 || { echo "$name failed"; tail -5 gpurun_out/$name.log; exit 1; }
done
echo ok

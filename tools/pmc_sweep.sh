#!/usr/bin/env bash
# PMC passes (one counter group per rocprofv3 run) over one frames.py workload.  GPU box only.
#   tools/pmc_sweep.sh NAME "frames.py args"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
name=$1; args=$2
i=0
for grp in "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_VALU GRBM_GUI_ACTIVE SQ_WAVES" "SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp -d gpurun_out/pmc_${name}_$i -o run --output-format csv -- python3 tools/frames.py --frames 1 $args > gpurun_out/pmc_${name}_$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc_${name}_$i.log; exit 1; }
done
echo ok

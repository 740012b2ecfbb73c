# round-6 final tree: rank 0's N-GPU share refreshed (C4 strong with bench.py's per-frame gather,
# without it, C3 weak), under the box's own 4 hardware queues
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_check.sh r06zi ranksharegather

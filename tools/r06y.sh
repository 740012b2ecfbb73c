# round-6: C3 at 20 steps: 3 in flight with batches on a partial grid (A/B)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
AB=c3pipe6 PASSES=4 bash tools/gpu_check.sh r06y ab

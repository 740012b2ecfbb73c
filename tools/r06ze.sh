# round-6: C3 with 3 contexts in flight on the full grid (A/B)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
AB=c3pipe7 PASSES=4 bash tools/gpu_check.sh r06ze ab

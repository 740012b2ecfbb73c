# round-6: the sphere room's pipeline, third sweep around 3 in flight with batches (A/B)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
AB=m2pipe8 PASSES=4 bash tools/gpu_check.sh r06x ab

# round-6: the sphere room's pipeline, second sweep around 3 in flight with batches (A/B)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
AB=m2pipe9 PASSES=6 bash tools/gpu_check.sh r06za ab

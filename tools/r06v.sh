# round-6: the sphere room's pipeline re-checked on the final kernels (A/B)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
AB=m2pipe6 PASSES=3 bash tools/gpu_check.sh r06v ab

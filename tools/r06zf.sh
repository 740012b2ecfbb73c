# round-6: kLegacyDefer re-swept on the batched sphere-room pipeline (A/B)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
AB=m2defer6 PASSES=4 bash tools/gpu_check.sh r06zf ab

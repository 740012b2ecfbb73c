# round-6 final tree: the N=8 share with gathers traced (hardware queues of render / gather /
# assembly kernels, overlap of consecutive frames)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_check.sh r06zj rstrace

# round-6 final tree: C5 brute force (the parity path), with gpu_check's heartbeat
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_check.sh r06zh benchc5

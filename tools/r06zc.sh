# round-6: mode 2's hit record with one normalize -- mode-2 parity + fuzz, then the A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_check.sh r06zc legacy fuzz || exit $?
AB=m2hitnorm PASSES=5 ABFIELD=ms_per_step,roofline.per_launch.kernel_ms bash tools/gpu_check.sh r06zc ab

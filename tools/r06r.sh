# round-6: mode 2's FAST sphere roots without the swap -- mode-2 parity + fuzz, then the A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_check.sh r06r legacy fuzz || exit $?
AB=m2roots PASSES=5 ABFIELD=ms_per_step,roofline.per_launch.kernel_ms bash tools/gpu_check.sh r06r ab

# round-6: the queue's tail grabs (debug library A/B)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
AB=tailgrab PASSES=3 ABFIELD=ms_per_step,roofline.per_launch.kernel_ms,config.frame_latency_ms_alone bash tools/gpu_check.sh r06p ab

# round-6: mode 2's dead marks -- mode-2 parity suites, then the A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_legacy.py tests/test_gpu_batch.py tests/test_gpu_spec_fuzz.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06o_pytest_m2.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r06o_pytest_m2.log
[ $rc -eq 0 ] || exit $rc
AB=m2dead PASSES=4 ABFIELD=ms_per_step,roofline.per_launch.kernel_ms,config.frame_latency_ms_alone bash tools/gpu_check.sh r06o ab

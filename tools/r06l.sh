# round-6: mode 2's spheres as literals -- mode-2 parity suites, then the A/B against the loop
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_legacy.py tests/test_gpu_batch.py tests/test_gpu_spec_fuzz.py tests/test_gpu_specialize.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r06l_pytest_m2.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r06l_pytest_m2.log
[ $rc -eq 0 ] || exit $rc
AB=m2slit PASSES=3 ABFIELD=ms_per_step,roofline.per_launch.kernel_ms,config.frame_latency_ms_alone bash tools/gpu_check.sh r06l ab

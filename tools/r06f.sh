set -o pipefail
DBG=rvcp-real-time-path-tracer_amd/csrc/build/librvcp_debug.so
RVCP_LIB=$DBG RVCP_DEBUG_TILE8=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_legacy.py tests/test_gpu_batch.py tests/test_gpu_parity.py tests/test_gpu_pipeline.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06f_pytest_tile8.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r06f_pytest_tile8.log
[ $rc -le 1 ] || exit $rc
AB=tile8 PASSES=3 ABFIELD=ms_per_step,roofline.per_launch.kernel_ms,config.interactive_ms_per_step bash tools/gpu_check.sh r06f ab

set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_legacy.py tests/test_gpu_batch.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06e_pytest_legacy.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r06e_pytest_legacy.log
[ $rc -le 1 ] || exit $rc
AB=m2order PASSES=3 ABFIELD=ms_per_step,roofline.per_launch.kernel_ms,config.interactive_ms_per_step bash tools/gpu_check.sh r06e ab && AB=steps20 PASSES=3 bash tools/gpu_check.sh r06e ab

set -o pipefail
bash tools/gpu_check.sh r06c ranksharegather rstrace pmcc3 && timeout -k 10 600 python -u -m pytest tests/test_gpu_specialize.py tests/test_gpu_bench.py -m gpu -x -v --timeout 280 --timeout-method thread > gpurun_out/r06c_pytest_spec_bench.log 2>&1; echo "pytest rc=$?"; tail -5 gpurun_out/r06c_pytest_spec_bench.log

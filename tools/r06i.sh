set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_spec_fuzz.py -m gpu -x -q --timeout 200 --timeout-method thread -k mode2 > gpurun_out/r06i_pytest_fuzz_mode2.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r06i_pytest_fuzz_mode2.log
[ $rc -le 1 ] || exit $rc
bash tools/gpu_check.sh r06i prof1

# round-6 re-entry: HEAD (mode-2 module changes) smoke + full GPU suite + the driver's command
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_check.sh r06q smoke tests || exit $?
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06q_bench_c3_driver.log 2>&1 || exit $?
grep '^{' gpurun_out/r06q_bench_c3_driver.log | tail -1 | cut -c1-400

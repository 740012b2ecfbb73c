# round-6: the sphere room's new automatic pipeline (bench line + the bench GPU tests), and
# mode 2 on the C3 frame with 3 in flight and batches (A/B)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --workload spheres --steps 60 --warmup 6 --no-cpu-baseline > gpurun_out/r06z_bench_spheres.log 2>&1 || exit $?
grep '^{' gpurun_out/r06z_bench_spheres.log | tail -1 | cut -c1-300
bash tools/gpu_check.sh r06z benchtest || exit $?
AB=c3m2pipe6 PASSES=3 bash tools/gpu_check.sh r06z ab

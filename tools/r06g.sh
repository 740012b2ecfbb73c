# round-6 evidence run on the final tree: smoke, the full GPU suite, the driver's bench command,
# the other workloads' bench lines, rocprofv3 kernel statistics of the headline command, the C3
# and sphere-room PMC passes (bound to this build), the N=2 self-launch rehearsal
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_check.sh r06g smoke tests || exit $?
b() {  # b <name> <limit> args...
    local name=$1 lim=$2; shift 2
    echo "=== bench $name ($(date +%T))"
    timeout -k 10 "$lim" python bench.py "$@" > "gpurun_out/r06g_bench_$name.log" 2>&1
    local rc=$?
    echo "=== bench $name rc=$rc"; grep '^{' "gpurun_out/r06g_bench_$name.log" | tail -1 | cut -c1-400
    [ $rc -le 1 ] || exit $rc
}
b c3_driver 300 --gpus 1 --steps 20 --warmup 5
b c3_60 300
b c2 300 --workload c2 --steps 100 --warmup 10
b spheres 300 --workload spheres --steps 60 --warmup 6 --no-cpu-baseline
b c3m2 300 --workload c3m2 --steps 40 --warmup 6 --no-cpu-baseline
b c4 300 --workload c4 --steps 10 --warmup 2 --no-cpu-baseline
b c6 300 --workload c6 --steps 20 --warmup 3 --no-cpu-baseline
b c5_bvh 300 --workload c5 --accel bvh --steps 12 --warmup 3 --no-cpu-baseline
b c3rot 300 --workload c3rot --steps 30 --warmup 5 --no-cpu-baseline
b c3gen 300 --workload c3gen --steps 30 --warmup 5 --no-cpu-baseline
bash tools/gpu_check.sh r06g prof pmcc3 spsqpmc spsqpmc2 selfl2

# round-6 final tree: smoke, the full GPU suite, the driver's bench command, C2 and the sphere
# room, one-frame rocprof stats, and the C3 / sphere-room PMC passes bound to this build
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_check.sh r06k smoke tests || exit $?
b() {  # b <name> <limit> args...
    local name=$1 lim=$2; shift 2
    echo "=== bench $name ($(date +%T))"
    timeout -k 10 "$lim" python bench.py "$@" > "gpurun_out/r06k_bench_$name.log" 2>&1
    local rc=$?
    echo "=== bench $name rc=$rc"; grep '^{' "gpurun_out/r06k_bench_$name.log" | tail -1 | cut -c1-300
    [ $rc -le 1 ] || exit $rc
}
bash tools/gpu_check.sh r06k pmcc3 spsqpmc spsqpmc2 prof1 || exit $?
b c3_driver 300 --gpus 1 --steps 20 --warmup 5
b c2 300 --workload c2 --steps 100 --warmup 10 --no-cpu-baseline
b spheres 300 --workload spheres --steps 60 --warmup 6 --no-cpu-baseline

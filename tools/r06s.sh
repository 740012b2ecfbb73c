# round-6 final tree: smoke, the full GPU suite, the C3 / sphere-room PMC passes bound to this
# build, one-frame rocprof stats, and every workload's bench line
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_check.sh r06s smoke tests || exit $?
b() {  # b <name> <limit> args...
    local name=$1 lim=$2; shift 2
    echo "=== bench $name ($(date +%T))"
    timeout -k 10 "$lim" python bench.py "$@" > "gpurun_out/r06s_bench_$name.log" 2>&1
    local rc=$?
    echo "=== bench $name rc=$rc"; grep '^{' "gpurun_out/r06s_bench_$name.log" | tail -1 | cut -c1-300
    [ $rc -le 1 ] || exit $rc
}
bash tools/gpu_check.sh r06s pmcc3 spsqpmc spsqpmc2 prof1 || exit $?
b c3_driver 300 --gpus 1 --steps 20 --warmup 5
b c2 300 --workload c2 --steps 100 --warmup 10 --no-cpu-baseline
b spheres 300 --workload spheres --steps 60 --warmup 6 --no-cpu-baseline
b c3m2 300 --workload c3m2 --steps 20 --warmup 3 --no-cpu-baseline
b c4 300 --workload c4 --steps 10 --warmup 2 --no-cpu-baseline
b c6 300 --workload c6 --steps 20 --warmup 3 --no-cpu-baseline
b c5_bvh 400 --workload c5 --steps 12 --warmup 3 --accel bvh --no-cpu-baseline
b c3rot 300 --workload c3rot --steps 30 --warmup 5 --no-cpu-baseline
b c3gen 300 --workload c3gen --steps 30 --warmup 5 --no-cpu-baseline
b c3_60 300

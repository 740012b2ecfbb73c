# round-6 final tree (after mode 2's hit-record change, which moves the build
# identity): smoke, the full GPU suite, the C3 / sphere-room PMC passes bound to this build,
# one-frame rocprof stats, the N=2 self-launch rehearsal and the headline bench lines
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_check.sh r06zd smoke tests || exit $?
bash tools/gpu_check.sh r06zd pmcc3 spsqpmc spsqpmc2 prof1 selfl2 || exit $?
b() {  # b <name> <limit> args...
    local name=$1 lim=$2; shift 2
    echo "=== bench $name ($(date +%T))"
    timeout -k 10 "$lim" python bench.py "$@" > "gpurun_out/r06zd_bench_$name.log" 2>&1
    local rc=$?
    echo "=== bench $name rc=$rc"; grep '^{' "gpurun_out/r06zd_bench_$name.log" | tail -1 | cut -c1-200
    [ $rc -le 1 ] || exit $rc
}
b c3_driver 300 --gpus 1 --steps 20 --warmup 5
b c2 300 --workload c2 --steps 100 --warmup 10 --no-cpu-baseline
b spheres 300 --workload spheres --steps 60 --warmup 6 --no-cpu-baseline
b c3m2 300 --workload c3m2 --steps 20 --warmup 3 --no-cpu-baseline
b c3_60 300

# round-6 final tree: the long rows measured again -- C5 brute force (the parity path; with its
# 128^2 SPP=1 CPU baseline) and c6 with the opt-in BVH
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
b() {  # b <name> <limit> args...
    local name=$1 lim=$2; shift 2
    echo "=== bench $name ($(date +%T))"
    timeout -k 10 "$lim" python bench.py "$@" > "gpurun_out/r06zg_bench_$name.log" 2>&1
    local rc=$?
    echo "=== bench $name rc=$rc"; grep '^{' "gpurun_out/r06zg_bench_$name.log" | tail -1 | cut -c1-300
    [ $rc -le 1 ] || exit $rc
}
b c6_bvh 300 --workload c6 --accel bvh --steps 20 --warmup 3 --no-cpu-baseline
b c5 900 --workload c5 --steps 1 --warmup 1

#!/usr/bin/env bash
# GPU-box check: build, smoke, gpu tests, bench, rocprofv3 kernel trace.
# Each GPU step has its own time limit; a fault/abort/timeout stops the script.
# Usage: tools/gpu_check.sh [tag] [steps...]   steps: smoke tests bench prof pmc
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r01}
shift || true
STEPS=${*:-"smoke tests bench prof"}
OUT=gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp

run() {  # run <name> <timeout> cmd...
    local name=$1 lim=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -n 25 "$OUT/$name.log"
    case $rc in
        0|1) return 0 ;;            # 1 = test failures / python error: keep going
        *) echo "STOP: $name exited $rc"; exit $rc ;;
    esac
}

echo "=== build"
python -c "import __graft_entry__ as g; g.build()" > "$OUT/build.log" 2>&1 || { tail -30 "$OUT/build.log"; exit 3; }
rocm-smi --showproductname > "$OUT/rocm-smi.txt" 2>&1 || true
lscpu > "$OUT/lscpu.txt" 2>&1 || true

for s in $STEPS; do
    case $s in
        smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
        tests) run pytest_gpu 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ;;
        newtests) run pytest_new 600 python -m pytest tests/test_golden_frames.py tests/test_interactive.py tests/test_scene_io.py tests/test_mandelbrot.py -m gpu -x -q ;;
        headless) run headless 300 python tools/headless.py --frames 120 --size 384 --spp 10 --dump gpurun_out/headless --format png --script walk ;;
        timeline) run timeline 300 bash -c "rm -f /tmp/tl.bin && RVCP_DEBUG_TIMELINE=/tmp/tl.bin python tools/frames.py --frames 3 && python tools/timeline.py /tmp/tl.bin --waves \$(python -c 'import os;print(os.path.getsize(\"/tmp/tl.bin\")//96)')" ;;
        timelinec2) run timelinec2 300 bash -c "rm -f /tmp/tl2.bin && RVCP_DEBUG_TIMELINE=/tmp/tl2.bin python tools/frames.py --frames 3 --size 384 --spp 10 && python tools/timeline.py /tmp/tl2.bin --waves \$(python -c 'import os;print(os.path.getsize(\"/tmp/tl2.bin\")//96)')" ;;
        timeline5) run timeline5 300 bash -c "rm -f /tmp/tl5.bin && RVCP_DEBUG_TIMELINE=/tmp/tl5.bin python tools/frames.py --variant 5 --frames 3 && python tools/timeline.py /tmp/tl5.bin --waves \$(python -c 'import os;print(os.path.getsize(\"/tmp/tl5.bin\")//96)')" ;;
        chunks) run chunks 500 bash -c "echo c3; python tools/frames.py --frames 10 || exit 1; echo c2; python tools/frames.py --frames 10 --size 384 --spp 10 || exit 1; echo sph; python tools/frames.py --integrator 1 --scene spheres --frames 10 --spp 5 || exit 1; echo small128; python tools/frames.py --frames 10 --size 128 --spp 30 || exit 1" ;;
        c5t) run c5t 400 bash -c "echo c5-512-v4; python tools/frames.py --variant 4 --frames 3 --tris 100000 --size 512 --spp 4 || exit 1; echo c5-512-v3; python tools/frames.py --variant 3 --frames 2 --tris 100000 --size 512 --spp 4" ;;
        w5) run w5 300 bash -c "echo c3-default; python tools/frames.py --frames 10 || exit 1; echo c3-w5; RVCP_LIB=rvcp-real-time-path-tracer_amd/csrc/build/variants/librvcp_w5.so python tools/frames.py --frames 10 || exit 1; echo c2-w5; RVCP_LIB=rvcp-real-time-path-tracer_amd/csrc/build/variants/librvcp_w5.so python tools/frames.py --frames 10 --size 384 --spp 10" ;;
        v35) run v35 900 bash -c "for v in 4 5 3; do echo c5 v\$v; python tools/frames.py --variant \$v --frames 2 --tris 100000 --size 512 --spp 4 || exit 1; done; for v in 3 5; do echo c3 v\$v; python tools/frames.py --variant \$v --frames 6 || exit 1; done; for v in 4 5; do echo c5-2k v\$v; python tools/frames.py --variant \$v --frames 2 --tris 2000 --size 512 --spp 8 || exit 1; done" ;;
        bvh) run pytest_bvh 600 python -m pytest tests/test_gpu_bvh.py -m gpu -x -q ;;
        bvhperf) run bvhperf 600 bash -c "echo c3-bvh; python tools/frames.py --frames 5 --accel 1 || exit 1; echo c5-bvh; python tools/frames.py --frames 3 --tris 100000 --accel 1 || exit 1" ;;
        legacy) run pytest_legacy 600 python -m pytest tests/test_gpu_legacy.py -m gpu -x -q ;;
        lframes) run lframes 300 python tools/frames.py --integrator 1 --scene spheres --frames 5 --spp 5 ;;
        bench) run bench 600 python bench.py --steps 20 --warmup 3 ;;
        bench2) run bench_c2 300 python bench.py --workload c2 --steps 50 --warmup 5 --no-cpu-baseline ;;
        rehearse2) run rehearse2 300 env RVCP_BENCH_REHEARSAL=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 5 --warmup 1 ;;
        rehearse4) run rehearse4 300 env RVCP_BENCH_REHEARSAL=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29532 bench.py --gpus 4 --steps 3 --warmup 1 ;;
        rcp) run rcp_check 120 tools/build/rcp_check ;;
        rcp2) run rcp_check2 300 tools/build/rcp_check2 ;;
        valu) run valu_rate 120 tools/build/valu_rate ;;
        pretest) run pretest_check 300 tools/build/pretest_check ;;
        c5small) run c5small 300 python tools/frames.py --variant 3 --frames 2 --tris 100000 --size 128 --spp 2 ;;
        c5cmp) run c5cmp 600 bash -c "python tools/frames.py --variant 4 --frames 2 --tris 100000 --size 512 --spp 4 && python tools/frames.py --variant 3 --frames 1 --tris 100000 --size 512 --spp 4" ;;
        prof) run prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$TAG" -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline ;;
        sqpmc) run sqpmc 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d "$OUT/sqpmc_$TAG" -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline ;;
        sqpmc2) run sqpmc2 600 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE -d "$OUT/sqpmc2_$TAG" -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline ;;
        c5pmc) run c5pmc 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d "$OUT/c5pmc_$TAG" -o run --output-format csv -- python3 tools/frames.py --frames 2 --tris 100000 --size 512 --spp 4 ;;
        c5pmc2) run c5pmc2 600 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_THREAD_CYCLES_VALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE -d "$OUT/c5pmc2_$TAG" -o run --output-format csv -- python3 tools/frames.py --frames 2 --tris 100000 --size 512 --spp 4 ;;
        listpmc) run listpmc 120 rocprofv3 -L ;;
        pmcf) run pmcf 600 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmcf_$TAG" -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline ;;
        pmcw) run pmcw 600 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmcw_$TAG" -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline ;;
        bvhvar) run bvhvar 900 bash -c 'for v in tools/build/var_*/librvcp.so; do echo "$v"; RVCP_LIB=$v python tools/frames.py --frames 2 --tris 100000 --accel 1 || exit 1; done' ;;
        c5var) run c5var 1100 bash -c 'for v in tools/build/var_*/librvcp.so; do echo "$v"; RVCP_LIB=$v python tools/frames.py --frames 2 --tris 100000 || exit 1; done' ;;
        benchc5bvh) run bench_c5_bvh 600 python bench.py --workload c5 --steps 3 --warmup 1 --accel bvh --no-cpu-baseline ;;
        benchc5) run bench_c5 900 python bench.py --workload c5 --steps 1 --warmup 1 ;;
        benchc4) run bench_c4 300 python bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline ;;
        c5pmcall) run c5pmcall 900 bash tools/c5_pmc.sh ;;
        benchc3m2) run bench_c3m2 300 python bench.py --workload c3m2 --steps 10 --warmup 2 --no-cpu-baseline ;;
        benchs) run bench_spheres 300 python bench.py --workload spheres --steps 50 --warmup 5 ;;
        profs) run profs 600 rocprofv3 --kernel-trace --stats -d "$OUT/profs_$TAG" -o run --output-format csv -- python3 bench.py --workload spheres --steps 20 --warmup 2 --no-cpu-baseline ;;
        abi) run pytest_abi 300 python -u -m pytest tests/test_gpu_abi.py -m gpu -x -v --timeout 120 --timeout-method thread ;;
        rehearse8c4) run rehearse8c4 400 env RVCP_BENCH_REHEARSAL=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29538 bench.py --gpus 8 --workload c4 --steps 5 --warmup 1 ;;
        rehearse2c4) run rehearse2c4 300 env RVCP_BENCH_REHEARSAL=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 1 ;;
        abpk) run abpk 600 bash -c 'bash tools/ab.sh "" packed scalar && bash tools/ab.sh "--size 384 --spp 10" packed scalar && bash tools/ab.sh "--size 2048 --spp 64 --frames 6" packed scalar' ;;
        configs) run pytest_configs 900 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -v --timeout 300 --timeout-method thread ;;
        valupmc) run valu_rate_wall 120 tools/build/valu_rate && run valupmc 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d "$OUT/valupmc_$TAG" -o run --output-format csv -- tools/build/valu_rate ;;
        calib) run calib_fetch 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/calibf_$TAG" -o run --output-format csv -- tools/build/traffic_calib && run calib_write 120 rocprofv3 --pmc WRITE_SIZE -d "$OUT/calibw_$TAG" -o run --output-format csv -- tools/build/traffic_calib ;;
        mtests) run pytest_m 600 python -u -m pytest tests/test_mandelbrot.py tests/test_golden_frames.py tests/test_gpu_configs.py -m gpu -x -v --timeout 300 --timeout-method thread ;;
        benchall) run bench_c3 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline && run bench_c2 300 python bench.py --workload c2 --steps 100 --warmup 10 --no-cpu-baseline && run bench_c4 300 python bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline ;;
        parity) run pytest_parity 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread ;;
        spreadab) run spreadab 600 bash tools/spread_ab.sh ;;
        spreadparity) run spreadparity 600 env RVCP_DEBUG_SPREAD=8 RVCP_DEBUG_EARLY_TAIL=1 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread ;;
        pmc) run pmc 600 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_$TAG" -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline ;;
    esac
done
echo "=== done"

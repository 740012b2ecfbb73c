#!/usr/bin/env bash
# GPU-box driver: smoke, GPU tests, benches, rocprofv3 kernel traces and PMC passes.  Each step
# runs under its own time limit; a fault / abort / timeout (rc >= 2) stops the script.  The
# libraries are built beforehand on the CPU (__graft_entry__.build()); nothing is built here
# except the tools' own checkers when a step needs them (tools/Makefile).
# Usage: tools/gpu_check.sh TAG step...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r03}
shift || true
STEPS=${*:-"smoke tests bench"}
TLARGS=${TLARGS:-}
OUT=gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
DBG=rvcp-real-time-path-tracer_amd/csrc/build/librvcp_debug.so

run() {  # run <name> <timeout> cmd...
    local name=$1 lim=$2; shift 2
    echo "=== $name ($(date +%T))"
    # heartbeat: a fresh box's first `import torch` can take minutes (the image pages in); the
    # step's own time limit, not silence, ends a step that hangs
    ( while sleep 60; do echo "    ... $name running ($(date +%T))"; done ) &
    local hb=$!
    timeout -k 10 "$lim" "$@" > "$OUT/${TAG}_$name.log" 2>&1
    local rc=$?
    kill $hb 2>/dev/null; wait $hb 2>/dev/null
    echo "=== $name rc=$rc"
    tail -n 25 "$OUT/${TAG}_$name.log"
    case $rc in
        0|1) return 0 ;;            # 1 = test failures / python error: keep going
        *) echo "STOP: $name exited $rc"; exit $rc ;;
    esac
}
tl() {  # per-wave timeline + in-kernel clock: tl <name> <frames> frames.py-args...
    local name=$1 nf=$2; shift 2
    run "$name" 300 bash -c "rm -f /tmp/tl_$name.bin && RVCP_LIB=$DBG RVCP_DEBUG_TIMELINE=/tmp/tl_$name.bin python tools/frames.py --frames $nf $* && python tools/timeline.py /tmp/tl_$name.bin --waves \$(python -c 'import os; print(os.path.getsize(\"/tmp/tl_$name.bin\") // 64 // $nf)')"
}

rocm-smi --showproductname > "$OUT/${TAG}_rocm-smi.txt" 2>&1 || true
for s in $STEPS; do
    case $s in
        smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
        tests) run pytest_gpu 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ;;
        parity) run pytest_parity 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_specialize.py -m gpu -x -q --timeout 300 --timeout-method thread ;;
        bvh) run pytest_bvh 600 python -u -m pytest tests/test_gpu_bvh.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread -k "bvh or BVH" ;;
        benchtest) run pytest_bench 600 python -u -m pytest tests/test_gpu_bench.py -m gpu -x -v --timeout 280 --timeout-method thread ;;
        rankshare) run rank_share 300 python -u tools/rank_share.py ;;
        # rank 0's share with bench.py's per-frame gather (world-1 RCCL
        # communicator attached as world N), under the box's own hardware queues; c4 strong and
        # c3 weak; and the N=8 share traced (queues of render, gather and assembly kernels)
        ranksharegather) run rank_share_c4 400 python -u tools/rank_share.py --workload c4 --gather && run rank_share_c4_nogather 400 python -u tools/rank_share.py --workload c4 --ns 2,4,8 && run rank_share_c3 400 python -u tools/rank_share.py --workload c3 --gather ;;
        rstrace) run rstrace 300 rocprofv3 --kernel-trace -d "$OUT/rstrace_$TAG" -o run --output-format csv -- python3 tools/rank_share.py --workload c4 --ns 8 --gather --frames 24 && python3 tools/trace_overlap.py "$OUT/rstrace_$TAG/run_kernel_trace.csv" --skip 6 >> "$OUT/${TAG}_rstrace.log" ;;
        # the four PMC passes of the headline command, for tools/pmc_valu.py / pmc_traffic.py
        # (--bench-log binds each summary to the build the passes ran)
        pmcc3) run sqpmc 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d "$OUT/sqpmc_$TAG" -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --interactive-pass 0 --frames-in-flight 1 --batch 1 && run sqpmc2 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE -d "$OUT/sqpmc2_$TAG" -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --interactive-pass 0 --frames-in-flight 1 --batch 1 && run pmcf 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmcf_$TAG" -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --interactive-pass 0 --frames-in-flight 1 --batch 1 && run pmcw 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmcw_$TAG" -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --interactive-pass 0 --frames-in-flight 1 --batch 1 ;;
        abi) run pytest_abi 300 python -u -m pytest tests/test_gpu_abi.py tests/test_gpu_specialize.py -m gpu -x -v --timeout 120 --timeout-method thread ;;
        bench) run bench_c3 600 python bench.py ;;
        benchq) run bench_c3q 300 python bench.py --steps 40 --warmup 5 --no-cpu-baseline ;;
        benchall) run bench_c3 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline && run bench_c2 300 python bench.py --workload c2 --steps 100 --warmup 10 --no-cpu-baseline && run bench_c4 300 python bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline ;;
        benchc4) run bench_c4 300 python bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline ;;
        benchc5) run bench_c5 900 python bench.py --workload c5 --steps 1 --warmup 1 ;;
        benchc5bvh) run bench_c5_bvh 600 python bench.py --workload c5 --steps 12 --warmup 3 --accel bvh --no-cpu-baseline ;;
        benchc3m2) run bench_c3m2 300 python bench.py --workload c3m2 --steps 20 --warmup 3 --no-cpu-baseline ;;
        benchs) run bench_spheres 300 python bench.py --workload spheres --steps 50 --warmup 5 --no-cpu-baseline ;;
        # the headline command under rocprofv3: default frames in flight, and one frame in flight
        # (per-launch durations that do not overlap -- roofline.per_launch)
        prof) run prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$TAG" -o run --output-format csv -- python3 bench.py --steps 60 --warmup 3 --no-cpu-baseline --interactive-pass 0 ;;
        # every launch timed (no warm-up, no launch pass): tools/trace_busy.py's busy time per frame,
# skipping the warm-up launches the bench reports (config.warmup_frames / frames_per_launch)
        profbusy) run profbusy 600 rocprofv3 --kernel-trace --stats -d "$OUT/profbusy_$TAG" -o run --output-format csv -- python3 bench.py --steps 20 --warmup 0 --launch-pass 0 --no-cpu-baseline --interactive-pass 0 && python3 tools/trace_busy.py "$OUT/profbusy_$TAG/run_kernel_trace.csv" --frames 20 --skip "$(python3 -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]['config']; print(-(-d['warmup_frames'] // d['frames_per_launch']))" "$OUT/${TAG}_profbusy.log")" >> "$OUT/${TAG}_profbusy.log" ;;
        # the reference's loop shape (1 frame per launch, 2 in flight) traced: do consecutive
        # frames' kernels overlap (tools/trace_overlap.py)?
        ovl) run ovl 300 rocprofv3 --kernel-trace -d "$OUT/ovl_$TAG" -o run --output-format csv -- python3 bench.py --steps 30 --warmup 0 --launch-pass 0 --no-cpu-baseline --interactive-pass 0 --frames-in-flight 2 --batch 1 ${OVLARGS:-} && python3 tools/trace_overlap.py "$OUT/ovl_$TAG/run_kernel_trace.csv" >> "$OUT/${TAG}_ovl.log" ;;
        ovli) run ovli 300 rocprofv3 --kernel-trace -d "$OUT/ovli_$TAG" -o run --output-format csv -- python3 bench.py --steps 8 --warmup 0 --launch-pass 0 --no-cpu-baseline --interactive-pass 20 ${OVLARGS:-} && python3 tools/trace_overlap.py "$OUT/ovli_$TAG/run_kernel_trace.csv" --last 20 >> "$OUT/${TAG}_ovli.log" ;;
        fifsweep) for f in 1 2 3 4; do run fif$f 300 python bench.py --steps 40 --warmup 4 --launch-pass 0 --no-cpu-baseline --interactive-pass 0 --frames-in-flight $f --batch 1 ${OVLARGS:-}; done ;;
        prof1) run prof1 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof1_$TAG" -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --interactive-pass 0 --frames-in-flight 1 --batch 1 ;;
        # PMC passes, one counter group per run (one frame in flight and one frame per launch, so
        # each dispatch is one frame of its own)
        pmcf) run pmcf 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmcf_$TAG" -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --interactive-pass 0 --frames-in-flight 1 --batch 1 ;;
        pmcw) run pmcw 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmcw_$TAG" -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --interactive-pass 0 --frames-in-flight 1 --batch 1 ;;
        sqpmc) run sqpmc 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d "$OUT/sqpmc_$TAG" -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --interactive-pass 0 --frames-in-flight 1 --batch 1 ;;
        sqpmc2) run sqpmc2 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE -d "$OUT/sqpmc2_$TAG" -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --interactive-pass 0 --frames-in-flight 1 --batch 1 ;;
        c5pmcf) run c5pmcf 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/c5pmcf_$TAG" -o run --output-format csv -- python3 bench.py --workload c5 --steps 1 --warmup 0 --launch-pass 0 --no-cpu-baseline --interactive-pass 0 --frames-in-flight 1 --batch 1 ;;
        c5pmcw) run c5pmcw 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/c5pmcw_$TAG" -o run --output-format csv -- python3 bench.py --workload c5 --steps 1 --warmup 0 --launch-pass 0 --no-cpu-baseline --interactive-pass 0 --frames-in-flight 1 --batch 1 ;;
        c5sqpmc) run c5sqpmc 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d "$OUT/c5sqpmc_$TAG" -o run --output-format csv -- python3 bench.py --workload c5 --steps 1 --warmup 0 --launch-pass 0 --no-cpu-baseline --interactive-pass 0 --frames-in-flight 1 --batch 1 ;;
        c5sqpmc2) run c5sqpmc2 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_THREAD_CYCLES_VALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE -d "$OUT/c5sqpmc2_$TAG" -o run --output-format csv -- python3 bench.py --workload c5 --steps 1 --warmup 0 --launch-pass 0 --no-cpu-baseline --interactive-pass 0 --frames-in-flight 1 --batch 1 ;;
        bvhsqpmc) run bvhsqpmc 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d "$OUT/bvhsqpmc_$TAG" -o run --output-format csv -- python3 bench.py --workload c5 --accel bvh --steps 2 --warmup 1 --launch-pass 0 --no-cpu-baseline --interactive-pass 0 --frames-in-flight 1 --batch 1 ;;
        bvhsqpmc2) run bvhsqpmc2 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE -d "$OUT/bvhsqpmc2_$TAG" -o run --output-format csv -- python3 bench.py --workload c5 --accel bvh --steps 2 --warmup 1 --launch-pass 0 --no-cpu-baseline --interactive-pass 0 --frames-in-flight 1 --batch 1 ;;
        m2sqpmc) run m2sqpmc 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d "$OUT/m2sqpmc_$TAG" -o run --output-format csv -- python3 bench.py --workload c3m2 --steps 5 --warmup 1 --no-cpu-baseline --interactive-pass 0 --frames-in-flight 1 --batch 1 ;;
        m2sqpmc2) run m2sqpmc2 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE -d "$OUT/m2sqpmc2_$TAG" -o run --output-format csv -- python3 bench.py --workload c3m2 --steps 5 --warmup 1 --no-cpu-baseline --interactive-pass 0 --frames-in-flight 1 --batch 1 ;;
        spsqpmc) run spsqpmc 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d "$OUT/spsqpmc_$TAG" -o run --output-format csv -- python3 bench.py --workload spheres --steps 10 --warmup 2 --no-cpu-baseline --interactive-pass 0 --frames-in-flight 1 --batch 1 ;;
        spsqpmc2) run spsqpmc2 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE -d "$OUT/spsqpmc2_$TAG" -o run --output-format csv -- python3 bench.py --workload spheres --steps 10 --warmup 2 --no-cpu-baseline --interactive-pass 0 --frames-in-flight 1 --batch 1 ;;
        # the chip's VALU issue ceiling and its in-kernel clock; the C3 kernel's in-kernel clock
        valu) run valu_rate 180 tools/build/valu_rate ;;
        valupmc) run valupmc 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d "$OUT/valupmc_$TAG" -o run --output-format csv -- tools/build/valu_rate ;;
        tlc3) tl tlc3 40 ;;
        tlreg) for k in 1 2 3 4 5; do run tlreg$k 300 bash -c "rm -f /tmp/tl_reg.bin && RVCP_LIB=$DBG RVCP_JIT_FLAGS=-DRVCP_REGION_CLOCK=$k RVCP_DEBUG_TIMELINE=/tmp/tl_reg.bin python tools/frames.py --frames 6 $TLARGS && python tools/timeline.py /tmp/tl_reg.bin --waves \$(python -c 'import os; print(os.path.getsize(\"/tmp/tl_reg.bin\") // 64 // 6)')"; done ;;
        tlc2) tl tlc2 40 --size 384 --spp 10 ;;
        rehearse2) run rehearse2 300 env RVCP_BENCH_REHEARSAL=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 5 --warmup 1 ;;
        frames) run frames 300 python tools/frames.py --frames 20 ;;
        # schedules 4 / 10 on meshes (tools/ab.py, one frame at a time)
        c5pool) run c5pool 900 python tools/ab.py --runner frames "s4=::--variant 4 --tris 2000 --size 1024 --spp 8 --frames 6" "s10=::--variant 10 --tris 2000 --size 1024 --spp 8 --frames 6" ;;
        spec) run pytest_spec 900 python -u -m pytest tests/test_gpu_specialize.py tests/test_gpu_pipeline.py tests/test_gpu_batch.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread ;;
        sqpmc3) run sqpmc3 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAVE_CYCLES -d "$OUT/sqpmc3_$TAG" -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --interactive-pass 0 --frames-in-flight 1 --batch 1 ;;
        sqrtchk) run sqrt_check 300 tools/build/sqrt_check ;;
        bvhtest) run pytest_bvh 600 python -u -m pytest tests/test_gpu_bvh.py -m gpu -x -v --timeout 300 --timeout-method thread ;;
        m2test) run pytest_m2 600 python -u -m pytest tests/test_gpu_legacy.py tests/test_gpu_specialize.py tests/test_gpu_batch.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread ;;
        benchsp) run bench_spheres 300 python bench.py --workload spheres --steps 60 --warmup 5 --no-cpu-baseline ;;
        tracec2) run tracec2 300 rocprofv3 --kernel-trace --stats -d "$OUT/tracec2_$TAG" -o run --output-format csv -- python3 tools/frames.py --size 384 --spp 10 --frames 30 ;;
        legacy) run pytest_legacy 600 python -u -m pytest tests/test_gpu_legacy.py tests/test_gpu_specialize.py -m gpu -x -q --timeout 300 --timeout-method thread ;;
        # same-box A/Bs: tools/ab_cases/$AB.txt (one case per line; the round's experiments are
        # recorded there with the variant libraries they compared, tools/build_variant.sh)
        ab) run ab_${AB} 900 python tools/ab.py --runner ${ABRUNNER:-bench} ${ABFIELD:+--field $ABFIELD} --passes ${PASSES:-3} --cases-file tools/ab_cases/${AB}.txt ;;
        pipeline) run pytest_pipeline 600 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_bench.py -m gpu -x -v --timeout 300 --timeout-method thread ;;
        benchrot) run bench_c3rot 300 python bench.py --workload c3rot --steps 30 --warmup 5 --no-cpu-baseline ;;
        benchgen) run bench_c3gen 300 python bench.py --workload c3gen --steps 30 --warmup 5 --no-cpu-baseline ;;
        benchc1) run bench_c1 300 python bench.py --workload c1 --steps 100 --warmup 10 ;;
        benchc2cpu) run bench_c2cpu 300 python bench.py --workload c2 --steps 100 --warmup 10 ;;
        # the driver's N>1 form without a launcher (bench.self_launch), one-GPU rehearsal
        selfl2) run selfl2 300 env RVCP_BENCH_REHEARSAL=1 python bench.py --gpus 2 --steps 10 --warmup 2 ;;
        c5tests) run c5tests 900 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "c5 or multi_tile or odd_remainder or variants or bitexact_cornell" ;;
        pooltests) run pooltests 600 python -u -m pytest tests/test_gpu_specialize.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread ;;
        fuzz) run pytest_fuzz 600 python -u -m pytest tests/test_gpu_spec_fuzz.py -m gpu -x -q --timeout 200 --timeout-method thread ;;
        spec2) run pytest_spec2 600 python -u -m pytest tests/test_gpu_specialize.py tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "not c5" ;;
        rccldiag) run rccl_diag 90 env RVCP_LIB=$DBG RVCP_DEBUG_RCCL_TRACE=1 NCCL_DEBUG=INFO NCCL_DEBUG_SUBSYS=INIT,BOOTSTRAP,ENV python -u tools/rccl_timeout_diag.py 3000 ;;
        abitest) run pytest_abi 300 python -u -m pytest tests/test_gpu_abi.py -m gpu -x -v --timeout 120 --timeout-method thread ;;
        rccltest) run pytest_rccl 300 python -u -m pytest tests/test_gpu_rccl_timeout.py tests/test_gpu_batch.py -m gpu -x -v --timeout 200 --timeout-method thread ;;
        c6test) run pytest_c6 900 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -v --timeout 600 --timeout-method thread -k c6 ;;
        benchc6) run bench_c6 300 python bench.py --workload c6 --steps 20 --warmup 3 ;;
        c6prof1) run c6prof1 300 rocprofv3 --kernel-trace --stats -d "$OUT/c6prof1_$TAG" -o run --output-format csv -- python3 bench.py --workload c6 --steps 4 --warmup 1 --no-cpu-baseline --interactive-pass 0 --frames-in-flight 1 --batch 1 ;;
        c6sqpmc) run c6sqpmc 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d "$OUT/c6sqpmc_$TAG" -o run --output-format csv -- python3 bench.py --workload c6 --steps 3 --warmup 1 --launch-pass 0 --no-cpu-baseline --interactive-pass 0 --frames-in-flight 1 --batch 1 ;;
        c6sqpmc2) run c6sqpmc2 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE -d "$OUT/c6sqpmc2_$TAG" -o run --output-format csv -- python3 bench.py --workload c6 --steps 3 --warmup 1 --launch-pass 0 --no-cpu-baseline --interactive-pass 0 --frames-in-flight 1 --batch 1 ;;
        *) echo "unknown step $s"; exit 2 ;;
    esac
done
echo "=== done"

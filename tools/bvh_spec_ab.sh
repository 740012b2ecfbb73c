#!/usr/bin/env bash
# speculative while-while BVH traversal (default) vs the if-if loop (RVCP_BVH_SPEC=0) and a
# count threshold (RVCP_BVH_SPEC_MIN=60): BVH parity of the product build, then C5 BVH frame time
set -e
timeout -k 5 300 python -u -m pytest tests/test_gpu_bvh.py tests/test_gpu_configs.py -m gpu -x -q --timeout 60 --timeout-method thread -k "bvh or BVH"
RVCP_LIB=tools/build/var_bvhspec60/librvcp.so timeout -k 5 150 python -u -m pytest tests/test_gpu_bvh.py -m gpu -x -q --timeout 60 --timeout-method thread
PASSES=${PASSES:-3} BENCH_ARGS="--workload c5 --accel bvh --steps 8 --warmup 2" timeout -k 10 900 bash tools/bench_ab.sh tools/build/var_bvhnospec/librvcp.so rvcp-real-time-path-tracer_amd/csrc/build/librvcp.so tools/build/var_bvhspec60/librvcp.so

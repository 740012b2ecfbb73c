#!/usr/bin/env bash
# packed-f32 slab fmas in the BVH node step (RVCP_BVH_PK=1 variant) vs the product build
set -e
V=tools/build/var_bvhpk/librvcp.so
RVCP_LIB=$V timeout -k 5 300 python -u -m pytest tests/test_gpu_bvh.py -m gpu -x -q --timeout 60 --timeout-method thread
PASSES=${PASSES:-3} BENCH_ARGS="--workload c5 --accel bvh --steps 8 --warmup 2" timeout -k 10 900 bash tools/bench_ab.sh rvcp-real-time-path-tracer_amd/csrc/build/librvcp.so $V

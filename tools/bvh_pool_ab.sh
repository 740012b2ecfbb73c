#!/usr/bin/env bash
# wave-pooled BVH traversal variants (RVCP_BVH_POOL=1; leaf chunk 2 / inlined) vs the product
# build: BVH parity of the leanest variant, then C5 BVH frame time, same box
set -e
RVCP_LIB=tools/build/var_bvhpoolc2in/librvcp.so timeout -k 5 300 python -u -m pytest tests/test_gpu_bvh.py tests/test_gpu_configs.py -m gpu -x -q --timeout 60 --timeout-method thread -k "bvh or BVH"
PASSES=${PASSES:-2} BENCH_ARGS="--workload c5 --accel bvh --steps 8 --warmup 2" timeout -k 10 900 bash tools/bench_ab.sh rvcp-real-time-path-tracer_amd/csrc/build/librvcp.so tools/build/var_bvhpool/librvcp.so tools/build/var_bvhpoolc2/librvcp.so tools/build/var_bvhpoolin/librvcp.so tools/build/var_bvhpoolc2in/librvcp.so

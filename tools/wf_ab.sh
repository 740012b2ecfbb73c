#!/usr/bin/env bash
# wavefront BVH path (default with --accel bvh) vs the persistent BVH path kernel (--schedule 3):
# BVH parity tests of both, then C5 BVH frame time, same box
set -e
timeout -k 5 300 python -u -m pytest tests/test_gpu_bvh.py tests/test_gpu_configs.py -m gpu -x -q --timeout 60 --timeout-method thread -k "bvh or BVH"
for pass in 1 2; do
  for sch in 3 0; do
    timeout -k 10 200 python bench.py --workload c5 --accel bvh --schedule $sch --steps 8 --warmup 2 --no-cpu-baseline --launch-pass 0 > /tmp/wfab.log 2>&1 || { tail -20 /tmp/wfab.log; exit 1; }
    python3 -c "
import json,sys; d=json.loads([l for l in open('/tmp/wfab.log') if l.startswith('{')][-1]); print('pass $pass schedule $sch ms_per_step %.2f Msamples/s %.1f fif %s' % (d['ms_per_step'], d['value'], d['config']['frames_in_flight']), flush=True)"
  done
done

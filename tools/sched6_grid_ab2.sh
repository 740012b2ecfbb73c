#!/bin/bash
# Schedule 6 (specialised, 6 waves/SIMD) vs 3: C3 / N=8 share at grid 2 and 3; C4 on one GPU
# (2 in flight, full grid).
set -o pipefail
for spec in 3:3 6:3 6:2 3:3 6:3 6:2; do
  IFS=: read -r v g <<< "$spec"
  line=$(timeout -k 10 200 python -u bench.py --steps 40 --warmup 4 --no-cpu-baseline --launch-pass 0 \
         --schedule $v --grid-waves $g 2>/dev/null | tail -1) || exit 1
  python -c "import json,sys; d=json.loads(sys.argv[1]); print('c3 schedule $v grid $g', d['ms_per_step'], flush=True)" "$line"
  timeout -k 10 200 python -u tools/rank_share.py --ns 8 --fif 3 --grid $g --schedule $v 2>/dev/null || exit 1
done
for v in 3 6 3 6; do
  line=$(timeout -k 10 200 python -u bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline --launch-pass 0 \
         --schedule $v 2>/dev/null | tail -1) || exit 1
  python -c "import json,sys; d=json.loads(sys.argv[1]); print('c4 schedule $v', d['ms_per_step'], d['config']['frames_in_flight'], d['config']['grid_waves_per_simd'], flush=True)" "$line"
done

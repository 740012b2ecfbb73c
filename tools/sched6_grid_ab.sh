#!/bin/bash
# The specialised 6-wave build (schedule 6) against the 5-wave one (3) under the C3-sized
# pipeline (3 frames in flight, grid_waves_per_simd G): C3 bench lines and the N=8 C4 share.
set -o pipefail
for spec in 3:3 6:3 6:4 3:3 6:3 6:4; do
  IFS=: read -r v g <<< "$spec"
  line=$(timeout -k 10 200 python -u bench.py --steps 40 --warmup 4 --no-cpu-baseline --launch-pass 0 \
         --schedule $v --grid-waves $g 2>/dev/null | tail -1) || exit 1
  python -c "import json,sys; d=json.loads(sys.argv[1]); print('c3 schedule $v grid $g', d['ms_per_step'], d['config']['kernel_schedule'], d['config']['scan'][:16], flush=True)" "$line"
  timeout -k 10 200 python -u tools/rank_share.py --ns 8 --fif 3 --grid $g --schedule $v 2>/dev/null || exit 1
done

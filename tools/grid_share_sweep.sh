#!/bin/bash
# Per-rank C4 shares (tools/rank_share.py) with the path kernel's persistent grid capped at B
# waves per SIMD (rvcp_config_t.grid_waves_per_simd) and F frames in flight: does a smaller
# grid per frame, with more frames beside it, shorten the serial-pixel tail of small shards
# ?  (profiles/r03zp_grid_share.log was taken with the debug build's grid cap,
# RVCP_DEBUG_BLOCKS_PER_CU, before the config field existed: the same launch geometry.)
#   tools/grid_share_sweep.sh "5 4 3 2" "2 3" "8,1" [extra rank_share.py args]
set -o pipefail
for f in ${2:-2 3}; do
  for b in ${1:-5 4 3}; do
    echo "== grid_waves_per_simd $b fif $f ${4:-}"
    timeout -k 10 200 python -u tools/rank_share.py --ns ${3:-8,1} --fif $f --frames 24 --grid $b \
        ${4:-} 2>/dev/null || exit 1
  done
done

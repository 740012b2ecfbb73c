set -e
cd $GRAFT_REPO_ROOT
RVCP_JIT_FLAGS="-DRVCP_DEBUG_COUNT_RESCAN" timeout -k 10 120 python tools/frames.py --frames 2 --size 1024 --spp 30 --variant 3
RVCP_NO_SPECIALIZE=1 timeout -k 10 120 python tools/frames.py --frames 2 --size 1024 --spp 30 --variant 3

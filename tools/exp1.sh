set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in base fma; do
  echo "== $v c3"; RVCP_LIB=tools/build/var_$v/librvcp.so timeout -k 10 120 python tools/frames.py --frames 10 | tail -3
  echo "== $v c5-512"; RVCP_LIB=tools/build/var_$v/librvcp.so timeout -k 10 200 python tools/frames.py --frames 2 --tris 100000 --size 512 --spp 4 | tail -1
done

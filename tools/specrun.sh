set -e
cd $GRAFT_REPO_ROOT
for v in base spec; do TAG=$v RVCP_LIB=tools/build/var_$v/librvcp.so timeout -k 10 120 python /root/repo/tools/cmpspec.py; done
python3 - <<'PY'
import numpy as np
for s in (1024, 384, 200):
    a = np.load(f"gpurun_out/spec_base_{s}.npy"); b = np.load(f"gpurun_out/spec_spec_{s}.npy")
    print(s, "bitexact", bool(np.array_equal(a.view(np.uint32), b.view(np.uint32))), int((a.view(np.uint32) != b.view(np.uint32)).sum()))
PY
bash tools/ab.sh "" base spec
bash tools/ab.sh "--size 384 --spp 10" base spec

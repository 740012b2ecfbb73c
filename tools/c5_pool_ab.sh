set -e
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_check.sh r03j c5tests
timeout -k 10 400 bash tools/sched_ab.sh "4 10" "--tris 100000 --size 512 --spp 4 --frames 5" "--tris 2000 --size 1024 --spp 8 --frames 6" "--tris 300 --size 1024 --spp 8 --frames 8" > gpurun_out/r03j_c5ab.log 2>&1
RVCP_LIB=tools/build/var_tpw4/librvcp.so timeout -k 10 300 bash tools/sched_ab.sh "10" "--tris 100000 --size 512 --spp 4 --frames 5" "--tris 2000 --size 1024 --spp 8 --frames 6" >> gpurun_out/r03j_c5ab.log 2>&1
for v in 4 10; do timeout -k 10 200 python tools/frames.py --variant $v --tris 100000 --size 1024 --spp 30 --frames 2 >> gpurun_out/r03j_c5ab.log 2>&1; done
cat gpurun_out/r03j_c5ab.log

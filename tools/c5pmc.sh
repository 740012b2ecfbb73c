set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 3
for v in 4 5; do
  timeout -k 10 300 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum -d gpurun_out/c5pmcA_v$v -o run --output-format csv -- python3 tools/frames.py --frames 1 --tris 100000 --spp 2 --variant $v > gpurun_out/c5pmcA_v$v.log 2>&1 || exit 4
  timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS -d gpurun_out/c5pmcB_v$v -o run --output-format csv -- python3 tools/frames.py --frames 1 --tris 100000 --spp 2 --variant $v > gpurun_out/c5pmcB_v$v.log 2>&1 || exit 5
done
echo done

# GPU box: k_nlist_wave with a rebuild every step (skin 0): kernel trace + one PMC pass
set -e
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/nl0
mkdir -p $OUT
cd /tmp
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-exact-compare --steps 10 --warmup 2 --neighbor-skin 0 > $OUT/prof.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR --kernel-include-regex k_nlist -d $OUT/pmc -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-exact-compare --steps 3 --warmup 1 --neighbor-skin 0 > $OUT/pmc.log 2>&1
cd $GRAFT_REPO_ROOT
python3 tools/pmc_show.py $OUT/pmc > $OUT/pmc.txt

#!/bin/bash
# round 4: matrix-pipe activity of k_g_spread_mfma (why its MFMAs do not hide behind the staging)
out=gpurun_out/r4ai
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
R=$GRAFT_REPO_ROOT
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --kernel-include-regex "k_g_spread|k_pairs_cq|k_g_interp" -d $R/$out/pmc -o run --output-format csv -- python3 $R/bench.py --kspace-algo 2 --no-cpu-baseline --no-exact-compare --steps 3 --warmup 1 > $R/$out/pmc.log 2>&1); step $? pmc
python3 tools/pmc_show.py $out/pmc | tee $out/pmc.txt

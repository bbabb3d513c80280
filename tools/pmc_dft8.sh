#!/bin/bash
# GPU box: PMC passes (separate runs) over the factorized DFT kernels of the C5 mixed bench
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_${1:-d8}
mkdir -p $OUT
cd /tmp
export TMPDIR=/tmp
B="$GRAFT_REPO_ROOT/bench.py --config C5 --precision mixed --no-cpu-baseline --no-exact-compare --no-kernel-timing --steps 2 --warmup 1"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex dft8 -d $OUT/f -o run --output-format csv -- python3 $B > $OUT/f.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex dft8 -d $OUT/w -o run --output-format csv -- python3 $B > $OUT/w.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --kernel-include-regex dft8 -d $OUT/a -o run --output-format csv -- python3 $B > $OUT/a.log 2>&1
cd $GRAFT_REPO_ROOT
for p in f w a; do python3 tools/pmc_show.py $OUT/$p; done > $OUT/summary.txt

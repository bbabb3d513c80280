#!/bin/bash
# Collect the round's rocprofv3 evidence for bench.py (C3) into gpurun_out/prof_<tag>/:
#   kernel trace + stats, and separate --pmc passes (MFMA/VALU/LDS activity, FETCH_SIZE,
#   WRITE_SIZE) as MI355X_MICROARCH.md prescribes.  Run on the GPU box from the repo root.
set -e
TAG=${1:-r01}
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG
ARGS="--steps 5 --warmup 2 --no-cpu-baseline --no-exact-compare"
mkdir -p $OUT
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS > $OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d $OUT/pmc_a -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS > $OUT/pmc_a.log 2>&1
timeout -k 10 300 rocprofv3 --pmc TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE -d $OUT/pmc_t -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS > $OUT/pmc_t.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_f -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS > $OUT/pmc_f.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_w -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS > $OUT/pmc_w.log 2>&1
cd $GRAFT_REPO_ROOT
python3 tools/pmc_summary.py $OUT/summary.json $OUT/trace/run_kernel_trace.csv $OUT/pmc_a/run_counter_collection.csv $OUT/pmc_t/run_counter_collection.csv $OUT/pmc_f/run_counter_collection.csv $OUT/pmc_w/run_counter_collection.csv > $OUT/summary.txt
cat $OUT/summary.txt

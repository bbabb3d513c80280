#!/bin/bash
# round 4: C5 mixed evidence at HEAD (after the tap-row and multi-round changes): kernel trace of
# the bench command and the FETCH / WRITE / SQ passes, summarized per kernel (pmc_summary.py).
out=gpurun_out/r4aq
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
R=$GRAFT_REPO_ROOT
ARGS="--config C5 --precision mixed --steps 5 --warmup 2 --no-cpu-baseline --no-exact-compare"
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$out/c5_trace -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/$out/c5_trace.log 2>&1); step $? c5_trace
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $R/$out/c5_pmc_f -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/$out/c5_pmc_f.log 2>&1); step $? c5_pmc_f
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $R/$out/c5_pmc_w -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/$out/c5_pmc_w.log 2>&1); step $? c5_pmc_w
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d $R/$out/c5_pmc_a -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/$out/c5_pmc_a.log 2>&1); step $? c5_pmc_a
python3 tools/pmc_summary.py $out/c5_summary.json $out/c5_trace/run_kernel_trace.csv $out/c5_pmc_a/run_counter_collection.csv $out/c5_pmc_f/run_counter_collection.csv $out/c5_pmc_w/run_counter_collection.csv > $out/c5_summary.txt 2>&1; head -16 $out/c5_summary.txt

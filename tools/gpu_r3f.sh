#!/bin/bash
# GPU session (round 3): new parity tests (interp2 vs interp, multi-rank overlap), isolated
# kernel times (CF_OVERLAP=0: one stream, so a kernel's duration is its own) of the new and the
# old spread / interpolation forms, and PMC passes of the new forms.  Each GPU step has its own
# time limit; the script stops at the first step that faults, aborts or times out.
out=gpurun_out/r3f
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_grid.py tests/test_gpu_overlap.py -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; echo "tests rc=$rc"; [ $rc -le 1 ] || exit $rc
R=$GRAFT_REPO_ROOT
ARGS="--steps 10 --warmup 3 --no-cpu-baseline --no-exact-compare"
cd /tmp && export TMPDIR=/tmp
export CF_OVERLAP=0
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$out/tr_new -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/$out/tr_new.log 2>&1; step $? tr_new
CF_SPREAD_DPP=0 CF_INTERP2=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$out/tr_old -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/$out/tr_old.log 2>&1; step $? tr_old
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d $R/$out/pmc_a -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/$out/pmc_a.log 2>&1; step $? pmc_a
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $R/$out/pmc_f -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/$out/pmc_f.log 2>&1; step $? pmc_f
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $R/$out/pmc_w -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/$out/pmc_w.log 2>&1; step $? pmc_w
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d $R/$out/cal_f -o run --output-format csv -- $R/tools/fetch_calib > $R/$out/cal_f.log 2>&1; step $? cal_f
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -d $R/$out/cal_w -o run --output-format csv -- $R/tools/fetch_calib > $R/$out/cal_w.log 2>&1; step $? cal_w
cd $R
python3 tools/fetch_calib.py $out/cal_f/run_counter_collection.csv $out/cal_w/run_counter_collection.csv $out/calibration.json
echo "== new (isolated)"; python3 tools/prof_stats.py $out/tr_new/run_kernel_stats.csv 14
echo "== old (isolated)"; python3 tools/prof_stats.py $out/tr_old/run_kernel_stats.csv 14
python3 tools/pmc_summary.py $out/summary.json $out/tr_new/run_kernel_trace.csv $out/pmc_a/run_counter_collection.csv $out/pmc_f/run_counter_collection.csv $out/pmc_w/run_counter_collection.csv > $out/summary.txt
head -12 $out/summary.txt | cut -c1-400
exit 0

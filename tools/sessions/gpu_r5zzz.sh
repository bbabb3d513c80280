#!/bin/bash
# round 5, third closing session at HEAD (after the pair kernel's phase-A rework, r05ah, and the
# energy kernel's block sums, r05al): full GPU suite, smoke, then per config the rocprofv3 kernel
# trace of the bench command and separate --pmc passes (VALU/LDS/wait counters, FETCH_SIZE,
# WRITE_SIZE) with the default (event) hand-over, whose summaries are copied into profiles/ as
# r05_c3/c5_pmc_summary_final.json BEFORE the bench lines run, so that the C3 and C5 bench lines'
# `traffic` is this build's.
out=gpurun_out/r5zzz
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
R=$GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1; step $? gpu_tests
tail -2 $out/gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1; step $? smoke
tail -3 $out/smoke.log
ARGS="--steps 5 --warmup 2 --no-cpu-baseline --no-exact-compare"
for cfg in c3 c5; do
  if [ $cfg = c5 ]; then CA="--config C5 --precision mixed"; else CA=""; fi
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$out/trace_$cfg -o run --output-format csv -- python3 $R/bench.py $ARGS $CA > $R/$out/trace_$cfg.log 2>&1); step $? trace_$cfg
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d $R/$out/pmc_a_$cfg -o run --output-format csv -- python3 $R/bench.py $ARGS $CA > $R/$out/pmc_a_$cfg.log 2>&1); step $? pmc_a_$cfg
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $R/$out/pmc_f_$cfg -o run --output-format csv -- python3 $R/bench.py $ARGS $CA > $R/$out/pmc_f_$cfg.log 2>&1); step $? pmc_f_$cfg
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $R/$out/pmc_w_$cfg -o run --output-format csv -- python3 $R/bench.py $ARGS $CA > $R/$out/pmc_w_$cfg.log 2>&1); step $? pmc_w_$cfg
  python3 tools/pmc_summary.py $out/summary_$cfg.json $out/trace_$cfg/run_kernel_trace.csv $out/pmc_a_$cfg/run_counter_collection.csv $out/pmc_f_$cfg/run_counter_collection.csv $out/pmc_w_$cfg/run_counter_collection.csv > $out/summary_$cfg.txt 2>&1; head -12 $out/summary_$cfg.txt
done
for cfg in c3 c5; do cp $out/summary_$cfg.json profiles/r05_${cfg}_pmc_summary_final.json; cp $out/summary_$cfg.txt profiles/r05_${cfg}_pmc_summary_final.txt; done
timeout -k 10 300 python -u bench.py > $out/bench_c3.json 2> $out/bench_c3.err; step $? bench_c3
timeout -k 10 300 python -u bench.py --config C5 --precision mixed --no-cpu-baseline > $out/bench_c5.json 2> $out/bench_c5.err; step $? bench_c5
python3 -c "
import json
for c in ('c3', 'c5'):
    d = json.loads(open('$out/bench_' + c + '.json').read().strip().splitlines()[-1])
    r = d['roofline']
    print(c, d['ms_per_step'], d['value'], d.get('ms_per_force_eval'), r['frac'], r.get('traffic'), r.get('traffic_source'), r.get('isolated', {}).get('avg_launch_ms'))"

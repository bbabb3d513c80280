#!/bin/bash
# round 4: full GPU suite at the cluster-pair default; eager vs hipGraph timelines (C3); rank-0
# scaling probe eager / graph; C5 mixed bench, trace and FETCH/WRITE passes.
out=gpurun_out/r4e
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1; rc=$?; tail -3 $out/gpu_tests.log; step $rc gpu_tests
R=$GRAFT_REPO_ROOT
for g in 0 1; do
    (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$out/tl_g$g -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-exact-compare --no-kernel-timing --graph $g > $R/$out/tl_g$g.log 2>&1); step $? tl_g$g
    python3 tools/trace_gaps.py $out/tl_g$g/run_kernel_trace.csv --steps 8
done
timeout -k 10 300 python -u tools/scaling_probe.py --worlds 1 8 --steps 40 --no-timing > $out/probe_eager.jsonl 2> $out/probe_eager.err; step $? probe_eager
timeout -k 10 300 python -u tools/scaling_probe.py --worlds 1 8 --steps 40 --graph > $out/probe_graph.jsonl 2> $out/probe_graph.err; step $? probe_graph
cat $out/probe_eager.jsonl $out/probe_graph.jsonl | cut -c1-200
timeout -k 10 600 python -u bench.py --config C5 --precision mixed --steps 10 --warmup 3 --no-cpu-baseline --no-exact-compare > $out/c5.json 2> $out/c5.err; step $? c5
python3 -c "import json; d=json.loads(open('$out/c5.json').read().strip().splitlines()[-1]); print('C5', d['ms_per_step'], d['ms_per_force_eval'], d['kernels_ms_per_step'])"
ARGS="--config C5 --precision mixed --steps 5 --warmup 2 --no-cpu-baseline --no-exact-compare"
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$out/c5_trace -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/$out/c5_trace.log 2>&1); step $? c5_trace
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $R/$out/c5_pmc_f -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/$out/c5_pmc_f.log 2>&1); step $? c5_pmc_f
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $R/$out/c5_pmc_w -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/$out/c5_pmc_w.log 2>&1); step $? c5_pmc_w
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d $R/$out/c5_pmc_a -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/$out/c5_pmc_a.log 2>&1); step $? c5_pmc_a
python3 tools/pmc_summary.py $out/c5_summary.json $out/c5_trace/run_kernel_trace.csv $out/c5_pmc_a/run_counter_collection.csv $out/c5_pmc_f/run_counter_collection.csv $out/c5_pmc_w/run_counter_collection.csv > $out/c5_summary.txt 2>&1; head -12 $out/c5_summary.txt

#!/bin/bash
# round 5, session ai: k_pairs_cq: the queue-length tests all_ge as one packed-byte scalar test (was
# v_mov/v_min3/v_min/v_cmp: 5 VALU per phase-B step and per batch), the fixed-range flag as a
# ballot accumulated in SGPRs (2 VALU fewer per pair).  Expected: SQ_INSTS_VALU 6.68e7 -> ~6.3e7,
# isolated 161 -> ~156 us.
out=gpurun_out/r5ai
mkdir -p $out
R=$GRAFT_REPO_ROOT
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_cluster.py tests/test_gpu_overlap.py tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_mixed.py tests/test_gpu_skin.py -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1; step $? tests
grep -E "passed|failed" $out/tests.log | tail -2
ARGS="--steps 40 --no-cpu-baseline --no-exact-compare"
for i in 1 2; do
  timeout -k 10 100 python -u bench.py $ARGS > $out/bench$i.json 2> $out/bench$i.err; step $? bench$i
  python3 -c "
import json; d = json.loads(open('$out/bench$i.json').read().strip().splitlines()[-1])
print('$i', d['ms_per_step'], d.get('graph_replay_ms_per_step'), round(d['roofline']['avg_launch_ms'], 4), d['roofline']['isolated']['avg_launch_ms'])"
done
A="--steps 5 --warmup 2 --no-cpu-baseline --no-exact-compare"
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/$out/trace -o run --output-format csv -- python3 $R/bench.py $A > $R/$out/trace.log 2>&1); step $? trace
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d $R/$out/pmc_a -o run --output-format csv -- python3 $R/bench.py $A > $R/$out/pmc_a.log 2>&1); step $? pmc_a
python3 tools/pmc_summary.py $out/summary_c3.json $out/trace/run_kernel_trace.csv $out/pmc_a/run_counter_collection.csv > $out/summary_c3.txt 2>&1; grep -E "pairs_cq" $out/summary_c3.txt
timeout -k 10 300 python -u bench.py --config C5 --precision mixed --no-cpu-baseline --no-exact-compare > $out/bench_c5.json 2> $out/bench_c5.err; step $? bench_c5
python3 -c "
import json; d = json.loads(open('$out/bench_c5.json').read().strip().splitlines()[-1])
print('c5', d['ms_per_step'], d.get('ms_per_force_eval'), d.get('graph_replay_ms_per_step'), d['roofline']['isolated']['avg_launch_ms'])"

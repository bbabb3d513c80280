#!/bin/bash
# round 5, session b (a repeated after a test bar fix): the option refactor (no CF_* environment), event hand-overs by default, and
# the interpolation's x-parity lane map (k_g_interp2: halo rows on disjoint LDS banks).
# Expected: k_g_interp2 SQ_LDS_BANK_CONFLICT / SQ_ACTIVE_INST_LDS 1.69 -> <= 0.3, isolated
# 77 -> ~60 us; a --pmc pass of bench.py completes with the default (event) hand-over;
# event vs memory hand-over step within ~2 %.
out=gpurun_out/r5b
# and k_pairs_cq with phase-B rows dealt to the fullest queues, the i side through the window:
# expected SQ_INSTS_VALU 7.5e7 -> ~6.2e7, isolated 184 -> ~155 us (bench breakdown direct_pairs).
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1; step $? gpu_tests
tail -2 $out/gpu_tests.log
timeout -k 10 300 python -u bench.py --steps 40 --no-cpu-baseline --no-exact-compare > $out/bench_event.json 2> $out/bench_event.err; step $? bench_event
timeout -k 10 300 python -u bench.py --steps 40 --no-cpu-baseline --no-exact-compare --handover memory > $out/bench_memory.json 2> $out/bench_memory.err; step $? bench_memory
python3 - <<'PY'
import json
for t in ("event", "memory"):
    d = json.loads(open(f"gpurun_out/r5b/bench_{t}.json").read().strip().splitlines()[-1])
    print(t, d["ms_per_step"], d["ms_per_force_eval"], d["graph_replay_ms_per_step"], {k: v for k, v in d["kernels_ms_per_step"].items() if v > 0.004})
PY
ARGS="--steps 5 --warmup 2 --no-cpu-baseline --no-exact-compare"
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$out/trace -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/$out/trace.log 2>&1); step $? trace
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d $R/$out/pmc_a -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/$out/pmc_a.log 2>&1); step $? pmc_a
python3 tools/pmc_summary.py $out/summary.json $out/trace/run_kernel_trace.csv $out/pmc_a/run_counter_collection.csv > $out/summary.txt 2>&1; head -30 $out/summary.txt

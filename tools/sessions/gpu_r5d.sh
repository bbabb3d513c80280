#!/bin/bash
# round 5, session d: k_pairs_cq back at the round-4 form (the row-dealing change of 81169b3 doubled it: 184 -> 374 us).
# The option refactor (event hand-overs by default), the interpolation x-parity lane map and
# k_pairs_cq with phase-B rows dealt to the fullest queues were committed without their GPU
# record surviving. Expected: suite green; k_g_interp2 conflicts/LDS-inst 1.69 -> <= 0.3;
# k_pairs_cq SQ_INSTS_VALU 7.5e7 -> ~6.2e7; a --pmc pass with the default hand-over completes.
out=gpurun_out/r5d
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_half.py tests/test_gpu_cluster.py tests/test_gpu_overlap.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1; step $? gpu_tests
tail -2 $out/gpu_tests.log
timeout -k 10 300 python -u bench.py --steps 40 --no-cpu-baseline --no-exact-compare > $out/bench_event.json 2> $out/bench_event.err; step $? bench_event
timeout -k 10 300 python -u bench.py --steps 40 --no-cpu-baseline --no-exact-compare --handover memory > $out/bench_memory.json 2> $out/bench_memory.err; step $? bench_memory
python3 - <<'PY'
import json
for t in ("event", "memory"):
    d = json.loads(open(f"gpurun_out/r5d/bench_{t}.json").read().strip().splitlines()[-1])
    print(t, d["ms_per_step"], d.get("ms_per_force_eval"), d.get("graph_replay_ms_per_step"), d.get("roofline"))
    print({k: v for k, v in d.get("kernels_ms_per_step", {}).items() if v > 0.004})
PY
ARGS="--steps 5 --warmup 2 --no-cpu-baseline --no-exact-compare"
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$out/trace -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/$out/trace.log 2>&1); step $? trace
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d $R/$out/pmc_a -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/$out/pmc_a.log 2>&1); step $? pmc_a
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $R/$out/pmc_f -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/$out/pmc_f.log 2>&1); step $? pmc_f
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $R/$out/pmc_w -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/$out/pmc_w.log 2>&1); step $? pmc_w
python3 tools/pmc_summary.py $out/summary.json $out/trace/run_kernel_trace.csv $out/pmc_a/run_counter_collection.csv $out/pmc_f/run_counter_collection.csv $out/pmc_w/run_counter_collection.csv > $out/summary.txt 2>&1; head -40 $out/summary.txt

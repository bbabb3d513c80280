#!/bin/bash
# round 5, session f: the octant (eighth-shell) cluster list, k_pairs_es (8-cell window, 512-thread
# blocks, two per CU).  Expected: octant tests green; k_pairs_es isolated <= k_pairs_cq (~184-209
# us) with the window writes 55 -> ~25 MB and k_excl 17 -> ~10 us.
out=gpurun_out/r5f
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_octant.py -x -v --timeout 120 --timeout-method thread > $out/gpu_tests.log 2>&1; step $? octant_tests
tail -3 $out/gpu_tests.log
ARGS="--steps 20 --no-cpu-baseline --no-exact-compare"
for pl in octant cluster; do
  timeout -k 10 120 python -u bench.py $ARGS --pair-list $pl > $out/bench_$pl.json 2> $out/bench_$pl.err; step $? bench_$pl
done
python3 - <<'PY'
import json
for t in ("octant", "cluster"):
    d = json.loads(open(f"gpurun_out/r5f/bench_{t}.json").read().strip().splitlines()[-1])
    print(t, d["ms_per_step"], d.get("ms_per_force_eval"), d.get("graph_replay_ms_per_step"), d["roofline"]["avg_launch_ms"], d["roofline"].get("isolated", {}).get("avg_launch_ms"))
    print({k: v for k, v in d.get("kernels_ms_per_step", {}).items() if v > 0.004})
PY
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/$out/trace -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-exact-compare > $R/$out/trace.log 2>&1); step $? trace
python3 tools/prof_stats.py $out/trace/run_kernel_stats.csv 2>/dev/null | head -30 || head -30 $out/trace/run_kernel_stats.csv

#!/bin/bash
# round 5, session ac: k_cl_build stages the cell's exclusion lists for all its i-clusters at once (the
# dependent gathers in flight block-wide), and the i-cluster boxes from LDS; k_cell_order with one
# 256-thread block per cell (was one wave).  Expected: k_cl_build 55 -> ~25-30 us, k_cell_order 25 -> ~8 us
# per rebuild (alone, breakdown pass), rebuild steps -20 us, C3 step -3..-5 us.
out=gpurun_out/r5ac
mkdir -p $out
R=$GRAFT_REPO_ROOT
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_cluster.py tests/test_gpu_half.py tests/test_gpu_octant.py tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_mixed.py -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1; step $? tests
grep -E "passed|failed" $out/tests.log | tail -1
ARGS="--steps 40 --no-cpu-baseline --no-exact-compare"
for i in 1 2 3; do
  timeout -k 10 100 python -u bench.py $ARGS > $out/bench$i.json 2> $out/bench$i.err; step $? bench$i
  python3 -c "
import json; d = json.loads(open('$out/bench$i.json').read().strip().splitlines()[-1])
print('c3', d['ms_per_step'], d.get('graph_replay_ms_per_step'), round(d['roofline']['avg_launch_ms'], 4), d['config'].get('nlist_builds_in_timed_steps'))"
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace -d $R/$out/trace -o run --output-format csv -- python3 $R/bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-exact-compare > $R/$out/trace.log 2>&1); step $? trace
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r5ac/trace/**/*kernel_trace.csv", recursive=True)[0]
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(f)))
d = [(e[1] - e[0]) / 1e3 for e in ev if "k_cl_build" in e[2]]
print("k_cl_build, breakdown pass (alone):", [round(x, 1) for x in d[5:45] if x > 5])
d = [(e[1] - e[0]) / 1e3 for e in ev if "k_cell_order" in e[2]]
print("k_cell_order, breakdown pass (alone):", [round(x, 1) for x in d[5:45]])
PY
python3 tools/step_stats.py $out/trace 46 85 | tail -2

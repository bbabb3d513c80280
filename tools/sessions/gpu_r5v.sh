#!/bin/bash
# round 5, session v: (1) device buffers zeroed at allocation, frees and graph-exec replacement
# only on an idle device, the fork / join stress test under changing flags (graph vs eager bits,
# builds == evaluations); (2) interpolation halo staging per x plane (k_g_interp2 staging VALU 248 ->
# 148 per wave: expected k_g_interp2 79 -> ~72 us, step -5 us), bitwise the same.
out=gpurun_out/r5v
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_overlap.py tests/test_gpu_grid.py -x -v --timeout 200 --timeout-method thread > $out/tests.log 2>&1; step $? tests
grep -E "passed|failed" $out/tests.log | tail -2
ARGS="--steps 40 --no-cpu-baseline --no-exact-compare"
for i in 1 2; do
  timeout -k 10 100 python -u bench.py $ARGS > $out/bench$i.json 2> $out/bench$i.err; step $? bench$i
  python3 -c "
import json; d = json.loads(open('$out/bench$i.json').read().strip().splitlines()[-1])
print('$i', d['ms_per_step'], d.get('graph_replay_ms_per_step'), round(d['roofline']['avg_launch_ms'], 4))"
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/trace -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-exact-compare > $GRAFT_REPO_ROOT/$out/trace.log 2>&1); step $? trace
python3 tools/step_timeline.py $out/trace | tail -12
grep -E "interp|spread_mfma|pairs_cq" $out/trace/run_kernel_stats.csv | cut -d, -f1-8

#!/bin/bash
# round 5, session x: graph mode with the event hand-overs recorded by event-record nodes inside
# the graphs (two graphs per evaluation instead of three).  Expected: C3 graph replay 0.47 -> ~0.45
# ms/step (= eager, as the memory form's two graphs measured in r05i), C5 graph 2.71 -> ~2.67;
# graph vs eager bits unchanged (test_gpu_graph, test_gpu_overlap).
out=gpurun_out/r5x
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_overlap.py -x -v --timeout 200 --timeout-method thread > $out/tests.log 2>&1; step $? tests
grep -E "passed|failed" $out/tests.log | tail -1
ARGS="--steps 40 --no-cpu-baseline --no-exact-compare"
for i in 1 2 3; do
  timeout -k 10 100 python -u bench.py $ARGS > $out/bench$i.json 2> $out/bench$i.err; step $? bench$i
  python3 -c "
import json; d = json.loads(open('$out/bench$i.json').read().strip().splitlines()[-1])
print('c3', d['ms_per_step'], d.get('graph_replay_ms_per_step'), round(d['roofline']['avg_launch_ms'], 4))"
done
timeout -k 10 300 python -u bench.py --config C5 --precision mixed --no-cpu-baseline > $out/bench_c5.json 2> $out/bench_c5.err; step $? bench_c5
python3 -c "
import json; d = json.loads(open('$out/bench_c5.json').read().strip().splitlines()[-1])
print('c5', d['ms_per_step'], d.get('ms_per_force_eval'), d.get('graph_replay_ms_per_step'))"

#!/bin/bash
# round 4: fork / join events with an agent-scope release (hipEventDisableSystemFence) against the
# default system-scope fence (CF_EVENT_FENCE=system): overlap / graph bitwise tests, one-step
# timelines eager and graph, alternated C3 benches, rank-0 probes W = 1 / 8 eager and graph.
out=gpurun_out/r4o
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_overlap.py tests/test_gpu_graph.py -x -q --timeout 150 --timeout-method thread > $out/tests.log 2>&1; rc=$?; tail -2 $out/tests.log; step $rc tests
for f in dev sys; do
    if [ $f = sys ]; then export CF_EVENT_FENCE=system; else unset CF_EVENT_FENCE; fi
    for g in 0 1; do
        (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$out/tl_${f}_g$g -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-exact-compare --no-kernel-timing --graph $g > $R/$out/tl_${f}_g$g.log 2>&1); step $? tl_${f}_g$g
        echo "$f graph=$g: $(python3 tools/trace_gaps.py $out/tl_${f}_g$g/run_kernel_trace.csv --steps 8)"
    done
done
for n in dev1 sys1 dev2 sys2; do
    if [ ${n%?} = sys ]; then export CF_EVENT_FENCE=system; else unset CF_EVENT_FENCE; fi
    timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-exact-compare > $out/bench_$n.json 2> $out/bench_$n.err; step $? bench_$n
    python3 -c "import json; d = json.loads(open('$out/bench_$n.json').read().strip().splitlines()[-1]); print('$n', d['ms_per_step'], d.get('graph_replay_ms_per_step'))"
done
unset CF_EVENT_FENCE
timeout -k 10 300 python -u tools/scaling_probe.py --worlds 1 8 --steps 40 --no-timing > $out/probe_eager.jsonl 2> $out/probe_eager.err; step $? probe_eager
timeout -k 10 300 python -u tools/scaling_probe.py --worlds 1 8 --steps 40 --graph > $out/probe_graph.jsonl 2> $out/probe_graph.err; step $? probe_graph
cat $out/probe_eager.jsonl $out/probe_graph.jsonl | cut -c1-150
python3 tools/step_timeline.py $out/tl_dev_g0 > $out/step_dev_g0.txt

#!/bin/bash
# round 4: fork / join by stream memory operations (default) against events (CF_SYNC=event):
# overlap / graph / multi-rank tests, one-step timelines, alternated C3 benches, rank-0 probes.
out=gpurun_out/r4q
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
R=$GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_gpu_overlap.py tests/test_gpu_graph.py tests/test_gpu_parity.py tests/test_gpu_skin.py -x -q --timeout 150 --timeout-method thread > $out/tests.log 2>&1; rc=$?; tail -2 $out/tests.log; step $rc tests
for v in val ev; do
    if [ $v = ev ]; then export CF_SYNC=event; else unset CF_SYNC; fi
    for g in 0 1; do
        (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$out/tl_${v}_g$g -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-exact-compare --no-kernel-timing --graph $g > $R/$out/tl_${v}_g$g.log 2>&1); step $? tl_${v}_g$g
        echo "$v graph=$g: $(python3 tools/trace_gaps.py $out/tl_${v}_g$g/run_kernel_trace.csv --steps 8)"
    done
    python3 tools/step_timeline.py $out/tl_${v}_g0 > $out/step_${v}_g0.txt
done
for n in val1 ev1 dax1 val2 ev2 dax2; do
    unset CF_SYNC CF_DIRECT_ON_AUX
    case $n in ev*) export CF_SYNC=event;; dax*) export CF_DIRECT_ON_AUX=1;; esac
    timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-exact-compare > $out/bench_$n.json 2> $out/bench_$n.err; step $? bench_$n
    python3 -c "import json; d = json.loads(open('$out/bench_$n.json').read().strip().splitlines()[-1]); print('$n', d['ms_per_step'], d.get('graph_replay_ms_per_step'))"
done
unset CF_SYNC CF_DIRECT_ON_AUX
timeout -k 10 300 python -u tools/scaling_probe.py --worlds 1 8 --steps 40 --no-timing > $out/probe_eager.jsonl 2> $out/probe_eager.err; step $? probe_eager
timeout -k 10 300 python -u tools/scaling_probe.py --worlds 1 8 --steps 40 --graph > $out/probe_graph.jsonl 2> $out/probe_graph.err; step $? probe_graph
cat $out/probe_eager.jsonl $out/probe_graph.jsonl | cut -c1-150

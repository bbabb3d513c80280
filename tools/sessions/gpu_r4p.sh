#!/bin/bash
# round 4: one rank's chains the other way round (CF_DIRECT_ON_AUX=1: the direct chain on the
# second stream, the reciprocal chain on the caller's) against the default: bitwise overlap tests,
# one-step timelines, alternated C3 benches (eager and graph).
out=gpurun_out/r4p
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
R=$GRAFT_REPO_ROOT
CF_DIRECT_ON_AUX=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_overlap.py tests/test_gpu_graph.py -x -q --timeout 150 --timeout-method thread > $out/tests.log 2>&1; rc=$?; tail -2 $out/tests.log; step $rc tests_dax
for v in base dax; do
    if [ $v = dax ]; then export CF_DIRECT_ON_AUX=1; else unset CF_DIRECT_ON_AUX; fi
    (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$out/tl_$v -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-exact-compare --no-kernel-timing > $R/$out/tl_$v.log 2>&1); step $? tl_$v
    echo "$v: $(python3 tools/trace_gaps.py $out/tl_$v/run_kernel_trace.csv --steps 8)"
    python3 tools/step_timeline.py $out/tl_$v > $out/step_$v.txt
done
for n in base1 dax1 hi1 base2 dax2 hi2; do
    unset CF_DIRECT_ON_AUX CF_AUX_PRIORITY
    case $n in dax*) export CF_DIRECT_ON_AUX=1;; hi*) export CF_AUX_PRIORITY=high;; esac
    timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-exact-compare > $out/bench_$n.json 2> $out/bench_$n.err; step $? bench_$n
    python3 -c "import json; d = json.loads(open('$out/bench_$n.json').read().strip().splitlines()[-1]); print('$n', d['ms_per_step'], d.get('graph_replay_ms_per_step'))"
done

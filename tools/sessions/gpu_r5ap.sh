#!/bin/bash
# round 5, session ap: a second full GPU suite + smoke + C3/C5 bench lines at HEAD on another box
# (stability of the late-round build before the driver's round-end runs).
out=gpurun_out/r5ap
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1; step $? gpu_tests
tail -1 $out/gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1; step $? smoke
timeout -k 10 300 python -u bench.py > $out/bench_c3.json 2> $out/bench_c3.err; step $? bench_c3
timeout -k 10 300 python -u bench.py --config C5 --precision mixed --no-cpu-baseline > $out/bench_c5.json 2> $out/bench_c5.err; step $? bench_c5
python3 -c "
import json
for c in ('c3', 'c5'):
    d = json.loads(open('$out/bench_' + c + '.json').read().strip().splitlines()[-1])
    print(c, d['ms_per_step'], d['value'], d.get('ms_per_force_eval'), d['roofline']['frac'], d.get('graph_replay_ms_per_step'))"

#!/bin/bash
# GPU session (round 3, final at HEAD after the r3q grid changes): the driver's commands -- full GPU test suite, smoke(),
# default bench line -- then the round's rocprofv3 evidence (tools/profile_round.sh r03u), the
# C5 mixed bench and the rank-0 scaling probe.  Each GPU step time-limited; stops at the first
# step that faults, aborts or times out.
out=gpurun_out/r3u
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; step $rc tests
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1; rc=$?; tail -2 $out/smoke.log; step $rc smoke
timeout -k 10 600 python -u bench.py > $out/bench.json 2> $out/bench.err; step $? bench
python - <<'P'
import json
d = json.loads(open("gpurun_out/r3u/bench.json").read().strip().splitlines()[-1])
print(d["value"], d["unit"], d["ms_per_step"], d["ms_per_force_eval"], d["roofline"]["avg_launch_ms"], d["roofline"]["frac"], d["cpu_baseline"]["value"])
P
timeout -k 10 1000 bash tools/profile_round.sh r03u > $out/profile_round.log 2>&1; step $? profile_round
tail -8 $out/profile_round.log | cut -c1-200
timeout -k 10 600 python -u bench.py --config C5 --precision mixed --steps 10 --warmup 3 --no-cpu-baseline --no-exact-compare > $out/bench_c5.json 2> $out/bench_c5.err; step $? bench_c5
timeout -k 10 300 python -u tools/scaling_probe.py --worlds 1 2 4 8 --no-timing --neighbor-skin 0.15 > $out/probe.json 2> $out/probe.err; step $? probe
cut -c1-100 $out/probe.json
exit 0

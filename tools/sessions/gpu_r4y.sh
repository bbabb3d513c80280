#!/bin/bash
# round 4: second-stream priority with the direct chain on it (CF_AUX_PRIORITY=high / low vs
# default): C3 benches, alternated, with the dominant launch's in-situ time.
out=gpurun_out/r4y
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
for n in def1 hi1 lo1 def2 hi2 lo2; do
    unset CF_AUX_PRIORITY
    case $n in hi*) export CF_AUX_PRIORITY=high;; lo*) export CF_AUX_PRIORITY=low;; esac
    timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-exact-compare > $out/bench_$n.json 2> $out/bench_$n.err; step $? bench_$n
    python3 -c "import json; d = json.loads(open('$out/bench_$n.json').read().strip().splitlines()[-1]); r = d['roofline']; print('$n', d['ms_per_step'], round(r['avg_launch_ms'], 4), r['frac'])"
done

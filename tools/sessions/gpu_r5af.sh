#!/bin/bash
# round 5, session af: grid kernel width W = 14 (default) against 12 and 10 at C3 (sigma 2 kept).
# Expected: spread and interpolation scale with W^3 where they are issue-bound (W = 12: -37 % taps),
# the k-space force error against the exact k-sum grows ~5x per width step (W = 14: 1e-8).
out=gpurun_out/r5af
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
for w in 14 12 10; do
  timeout -k 10 200 python -u bench.py --steps 40 --no-cpu-baseline --grid-width $w > $out/exact_w$w.json 2> $out/exact_w$w.err; step $? exact_w$w
  python3 -c "
import json; d = json.loads(open('$out/exact_w$w.json').read().strip().splitlines()[-1])
print('exact $w', d['ms_per_step'], json.dumps(d.get('exact_kspace'))[:300]); print(json.dumps(d.get('kernels_ms_per_step'))[:900])"
done
ARGS="--steps 40 --no-cpu-baseline --no-exact-compare"
for w in 14 12 10 14 12 10; do
  timeout -k 10 100 python -u bench.py $ARGS --grid-width $w > $out/bench_w$w.json 2> $out/bench_w$w.err; step $? w$w
  python3 -c "
import json; d = json.loads(open('$out/bench_w$w.json').read().strip().splitlines()[-1])
print('c3 $w', d['ms_per_step'], d.get('graph_replay_ms_per_step'), d['config'].get('kspace'))"
done

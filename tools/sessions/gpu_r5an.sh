#!/bin/bash
# round 5, session an: neighbour-skin re-sweep with the cluster-pair list (the defaults 0.15 C3 /
# 0.2 C5 date from round 2's per-atom lists, whose build cost 4x more).  A smaller skin shrinks the
# list (phase-A tests per pair ~ (rc + skin)^3) and rebuilds more often (k_cl_build 32 us C3 /
# 133 us C5 per build).  Expected: C5 optimum at 0.1-0.15 (-50..-100 us per step), C3 within +-5 us.
out=gpurun_out/r5an
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
for sk in 0.2 0.15 0.125 0.1 0.2 0.15 0.125 0.1; do
  timeout -k 10 200 python -u bench.py --config C5 --precision mixed --steps 40 --no-cpu-baseline --no-exact-compare --neighbor-skin $sk > $out/c5_$sk.json 2> $out/c5_$sk.err; step $? c5_$sk
  python3 -c "
import json; d = json.loads(open('$out/c5_$sk.json').read().strip().splitlines()[-1])
print('c5 $sk', d['ms_per_step'], d['config']['nlist_builds_in_timed_steps'], d['kernels_ms_per_step']['direct_pairs'], d['kernels_ms_per_step']['neighbor_list'])"
done
for sk in 0.15 0.125 0.1 0.15 0.125 0.1; do
  timeout -k 10 100 python -u bench.py --steps 40 --no-cpu-baseline --no-exact-compare --neighbor-skin $sk > $out/c3_$sk.json 2> $out/c3_$sk.err; step $? c3_$sk
  python3 -c "
import json; d = json.loads(open('$out/c3_$sk.json').read().strip().splitlines()[-1])
print('c3 $sk', d['ms_per_step'], d['config']['nlist_builds_in_timed_steps'], d['kernels_ms_per_step']['direct_pairs'], d['kernels_ms_per_step']['neighbor_list'])"
done

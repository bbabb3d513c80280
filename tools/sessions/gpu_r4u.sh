#!/bin/bash
# round 4: neighbour-skin sweep at C3 for the cluster-pair list (its build is ~2x cheaper than the
# per-atom list's, so the round-2 optimum 0.15 nm may have moved), two passes.
out=gpurun_out/r4u
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
for p in 1 2; do
    for sk in 0.06 0.08 0.10 0.12 0.15; do
        timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-exact-compare --neighbor-skin $sk > $out/bench_${sk}_$p.json 2> $out/bench_${sk}_$p.err; step $? bench_${sk}_$p
        python3 -c "import json; d = json.loads(open('$out/bench_${sk}_$p.json').read().strip().splitlines()[-1]); k = d['kernels_ms_per_step']; print('skin $sk pass $p', d['ms_per_step'], k['direct_pairs'], k['neighbor_list'], k['cell_sort'])"
    done
done

#!/bin/bash
# round 5, session ao: cells sized for a 0.2 nm skin (16^3 at C5) while the list uses a smaller
# skin (temporary variant bit 12).  r05an: a smaller skin at C5 made the pair kernel slower because
# the cells shrank (16^3 -> 17^3); keeping 16^3 cells, skin 0.15 / 0.125 should cut phase-A tests
# by 12 / 17 % (list volume).  Expected: C5 pair kernel 1.25 -> ~1.15 ms, step -60..-90 us net of
# the extra rebuilds.
out=gpurun_out/r5ao
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
for cfg in "0.2 0" "0.15 4096" "0.125 4096" "0.1 4096" "0.2 0" "0.15 4096" "0.125 4096" "0.1 4096"; do
  set -- $cfg; sk=$1; v=$2
  timeout -k 10 200 python -u bench.py --config C5 --precision mixed --steps 40 --no-cpu-baseline --no-exact-compare --neighbor-skin $sk --variants $v > $out/c5_${sk}_$v.json 2> $out/c5_${sk}_$v.err; step $? c5_$sk
  python3 -c "
import json; d = json.loads(open('$out/c5_${sk}_$v.json').read().strip().splitlines()[-1])
print('c5 $sk $v', d['ms_per_step'], d['config']['nlist_builds_in_timed_steps'], d['kernels_ms_per_step']['direct_pairs'], d['kernels_ms_per_step']['neighbor_list'], d['energy_kj_mol'])"
done

#!/bin/bash
# round 5, session ar: the C3 bench line with its new default skin 0.125 (r05an: -3.4 us per step
# against 0.15 on one box, 8^3 cells either way), against --neighbor-skin 0.15, alternating.
out=gpurun_out/r5ar
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
for a in "d" "0.15" "d" "0.15" "d" "0.15"; do
  if [ $a = d ]; then X=""; else X="--neighbor-skin $a"; fi
  timeout -k 10 100 python -u bench.py --steps 40 --no-cpu-baseline --no-exact-compare $X > $out/c3_$a.json 2> $out/c3_$a.err; step $? c3_$a
  python3 -c "
import json; d = json.loads(open('$out/c3_$a.json').read().strip().splitlines()[-1])
print('c3 $a', d['config']['neighbor_skin_nm'], d['ms_per_step'], d['config']['nlist_builds_in_timed_steps'], d['kernels_ms_per_step']['direct_pairs'])"
done
timeout -k 10 300 python -u bench.py > $out/bench_c3.json 2> $out/bench_c3.err; step $? bench_c3
python3 -c "
import json; d = json.loads(open('$out/bench_c3.json').read().strip().splitlines()[-1])
print('c3 default line', d['ms_per_step'], d['value'], d['roofline']['frac'], d['config']['neighbor_skin_nm'], d['cpu_baseline']['value'])"

#!/bin/bash
# round 5, session am: schedule A/B -- the pair kernel gated on the forward DFT (variant bit 12,
# temporary, eager only) so that the coefficients, inverse DFT and interpolation run beside the
# pair kernel instead of after it (today the x-stage, coefficients, inverse DFT, interpolation and
# energy, ~150 us, are exposed after the pair kernel).  Expected: C3 -10..+10 us (the pair kernel
# starts ~40 us later; the tail shrinks if the interpolation gets CUs between pair blocks).
out=gpurun_out/r5am
mkdir -p $out
R=$GRAFT_REPO_ROOT
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
ARGS="--steps 40 --no-cpu-baseline --no-exact-compare"
for v in 0 4096 0 4096 0 4096; do
  timeout -k 10 100 python -u bench.py $ARGS --variants $v > $out/bench_$v.json 2> $out/bench_$v.err; step $? bench_$v
  python3 -c "
import json; d = json.loads(open('$out/bench_$v.json').read().strip().splitlines()[-1])
print('c3 $v', d['ms_per_step'], d['energy_kj_mol'], round(d['roofline']['avg_launch_ms'], 4))"
done
A="--steps 5 --warmup 2 --no-cpu-baseline --no-exact-compare --variants 4096"
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/$out/trace -o run --output-format csv -- python3 $R/bench.py $A > $R/$out/trace.log 2>&1); step $? trace
python3 tools/step_timeline.py $out/trace | tail -30

#!/bin/bash
# round 5, session p: CF_VARIANT_PAIR_TAIL n (variants bits 12-21): the last n of the 512 C3 cells of
# the pair kernel are launched after the spread (they then run beside the DFT stages, whose launches
# otherwise wait ~90-185 us for pair blocks to end, and the interpolation).  Expected: n = 128-256
# step -10..-40 us.  Plus the bitwise check of the split (overlap test) through the variant.
out=gpurun_out/r5p
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
ARGS="--steps 40 --no-cpu-baseline --no-exact-compare"
for n in 0 128 192 256 320 0 128 192 256 320; do
  timeout -k 10 100 python -u bench.py $ARGS --variants $(( n << 12 )) > $out/bench_t$n.json 2> $out/bench_t$n.err; step $? t$n
  python3 -c "
import json; d = json.loads(open('$out/bench_t$n.json').read().strip().splitlines()[-1])
print('$n', d['ms_per_step'], d.get('graph_replay_ms_per_step'), round(d['roofline']['avg_launch_ms'], 4), d['config'].get('fp64_rescan_fallbacks_in_timed_steps'))"
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/$out/trace192 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-exact-compare --variants $(( 192 << 12 )) > $GRAFT_REPO_ROOT/$out/trace192.log 2>&1); step $? trace192
python3 tools/step_timeline.py $out/trace192 | tail -28

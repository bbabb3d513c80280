#!/bin/bash
# round 5, session r: HIP stream priority of the second stream (the direct chain: cell list, pair
# kernel, exclusions) -- variants bits 12-13: 1 = lowest, 2 = highest, 0 = normal.  Expected with
# the lowest: the DFT stages get the CUs the pair kernel's first-round blocks free (zfwd ~99 us under
# the pair kernel today), the interpolation overlaps the pair kernel's second round: step -20..-80 us.
out=gpurun_out/r5r
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
ARGS="--steps 40 --no-cpu-baseline --no-exact-compare"
for v in 0 4096 8192 0 4096 8192; do
  timeout -k 10 100 python -u bench.py $ARGS --variants $v > $out/bench_v$v.json 2> $out/bench_v$v.err; step $? v$v
  python3 -c "
import json; d = json.loads(open('$out/bench_v$v.json').read().strip().splitlines()[-1])
print('$v', d['ms_per_step'], d.get('graph_replay_ms_per_step'), round(d['roofline']['avg_launch_ms'], 4))"
done
head -2 $out/bench_v4096.err
for v in 4096 8192; do
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/$out/trace$v -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-exact-compare --variants $v > $GRAFT_REPO_ROOT/$out/trace$v.log 2>&1); step $? trace$v
python3 tools/step_timeline.py $out/trace$v | tail -20
done

#!/bin/bash
# round 5, session q: the interpolation over runs of x-adjacent tiles (k_g_interp2s, a ring of
# halo x planes: 8 of 21 planes staged per tile after the first, prefetched during the previous
# tile's atoms).  Expected: k_g_interp2s 78 -> ~60 us per launch (staging VALU 6.4e6 -> ~2.5e6,
# L2->LDS halo traffic 303 -> ~140 MB), step -10..-20 us; bitwise equal to the tile kernel.
out=gpurun_out/r5q
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_grid.py -k "interp" -x -v --timeout 120 --timeout-method thread > $out/tests.log 2>&1; step $? tests
tail -3 $out/tests.log
ARGS="--steps 40 --no-cpu-baseline --no-exact-compare"
for v in 0 32 16384 0 32 16384; do
  timeout -k 10 100 python -u bench.py $ARGS --variants $v > $out/bench_v$v.json 2> $out/bench_v$v.err; step $? v$v
  python3 -c "
import json; d = json.loads(open('$out/bench_v$v.json').read().strip().splitlines()[-1])
print('$v', d['ms_per_step'], d.get('graph_replay_ms_per_step'), round(d['roofline']['avg_launch_ms'], 4))"
done
for v in 0 32; do
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/trace$v -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-exact-compare --variants $v > $GRAFT_REPO_ROOT/$out/trace$v.log 2>&1); step $? trace$v
python3 tools/step_timeline.py $out/trace$v | tail -14
done

#!/bin/bash
# round 5, session m: the cluster-pair loop issued as p launches over consecutive cell ranges
# (CF_VARIANT_PAIR_PARTS p = variants bits 12-14): a pair block holds its CU ~90 us, so the DFT
# stages queued behind the spread wait for the whole pair launch (r5f/r5k timelines); with p
# launches each ends sooner.  Expected: p = 2..4 step -10..-40 us, or nothing.
out=gpurun_out/r5m
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_mixed.py tests/test_gpu_half.py -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1; step $? tests
tail -2 $out/gpu_tests.log
ARGS="--steps 40 --no-cpu-baseline --no-exact-compare"
for p in 1 2 4 3; do
  timeout -k 10 100 python -u bench.py $ARGS --variants $(( p << 12 )) > $out/bench_p$p.json 2> $out/bench_p$p.err; step $? p$p
  python3 -c "
import json; d = json.loads(open('$out/bench_p$p.json').read().strip().splitlines()[-1])
print('$p', d['ms_per_step'], d.get('graph_replay_ms_per_step'), round(d['roofline']['avg_launch_ms'], 4), d['config'].get('fp64_rescan_fallbacks_in_timed_steps'))"
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/$out/trace2 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-exact-compare --variants $(( 2 << 12 )) > $GRAFT_REPO_ROOT/$out/trace2.log 2>&1); step $? trace2
python3 tools/step_timeline.py $out/trace2 | tail -28

#!/bin/bash
# round 5, session aa: per-step order of the two chains in the timed region (rocprofv3 kernel trace
# of bench.py --steps 40 --warmup 5; steps 46-85 are the timed ones).  Question: in steps that keep
# the list, does k_pairs_cq start before the grid bin sort / spread and starve them (traced short
# runs: g_bin 80-115 us instead of 11, step ~515 us against ~455 on rebuild steps)?
out=gpurun_out/r5aa
mkdir -p $out
R=$GRAFT_REPO_ROOT
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace -d $R/$out/trace -o run --output-format csv -- python3 $R/bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-exact-compare > $R/$out/trace.log 2>&1); rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/step_stats.py $out/trace 46 85 | tail -45
# A/B: the pair kernel gated on the grid bin sort (variants 1 << 12) or on the spread (2 << 12);
# expected if the kept-list steps are starved as traced: -20..-50 us per such step
ARGS="--steps 40 --no-cpu-baseline --no-exact-compare"
for v in 0 4096 8192 0 4096 8192; do
  timeout -k 10 100 python -u bench.py $ARGS --variants $v > $out/bench_v$v.json 2> $out/bench_v$v.err; rc=$?; echo "v$v rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 -c "
import json; d = json.loads(open('$out/bench_v$v.json').read().strip().splitlines()[-1])
print('$v', d['ms_per_step'], d.get('ms_per_force_eval'), round(d['roofline']['avg_launch_ms'], 4), d['config'].get('nlist_builds_in_timed_steps'))"
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace -d $R/$out/trace_g1 -o run --output-format csv -- python3 $R/bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-exact-compare --variants 4096 > $R/$out/trace_g1.log 2>&1); rc=$?; echo "trace_g1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/step_stats.py $out/trace_g1 46 85 | tail -3

#!/bin/bash
# round 5, session o: (1) the exp polynomial's constants as SGPR operands (the fp64 pair kernels
# had 32-40 B/lane of spills, none now; bitwise the same arithmetic); (2) the persistent pair
# kernel leaving n CUs to the reciprocal chain (CF_VARIANT_PAIR_FREE_CUS n, variants bits 12-18),
# now with few spills (r5k: 96 B/lane, isolated 198 us).  Expected: default isolated 181 -> ~175 us;
# n = 32-64: the DFT stages beside the pair kernel, step -10..-40 us.
out=gpurun_out/r5o
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
timeout -k 10 500 python -u -m pytest tests/test_gpu_cluster.py tests/test_gpu_overlap.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $out/gpu_tests.log 2>&1; step $? tests
tail -2 $out/gpu_tests.log
ARGS="--steps 40 --no-cpu-baseline --no-exact-compare"
for n in 0 32 48 64 0 32 48 64; do
  timeout -k 10 100 python -u bench.py $ARGS --variants $(( n << 12 )) > $out/bench_n$n.json 2> $out/bench_n$n.err; step $? n$n
  python3 -c "
import json; d = json.loads(open('$out/bench_n$n.json').read().strip().splitlines()[-1])
print('$n', d['ms_per_step'], d.get('graph_replay_ms_per_step'), round(d['roofline']['avg_launch_ms'], 4), round(d['roofline']['isolated']['avg_launch_ms'], 4), d['config'].get('fp64_rescan_fallbacks_in_timed_steps'))"
done

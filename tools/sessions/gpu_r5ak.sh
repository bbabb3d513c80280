#!/bin/bash
# round 5, session ak: same-box A/B after r05aj (the packed-byte all_ge made k_pairs_cq slower:
# C5 pair kernel 1.266 -> 1.326 ms).  A = ba119e2, F = A + ballot fixed-range flag + degree-10 exp
# polynomial (each neutral-to-faster in r05aj), G = F with the room check back in vector form
# (tests whether r05ah's packed-byte room check costs the same way).  Expected: F <= A by 1-2 us
# isolated; G vs F decides the room check.
out=gpurun_out/r5ak
mkdir -p $out
L=openmm-chargeflux_amd/libchargeflux_hip.so
cp $L $out/lib_orig.so
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
ARGS="--steps 40 --no-cpu-baseline --no-exact-compare"
for v in A F G A F G; do
  cp tools/ab/lib_$v.so $L
  timeout -k 10 100 python -u bench.py $ARGS > $out/bench_$v.json 2> $out/bench_$v.err; step $? bench_$v
  python3 -c "
import json; d = json.loads(open('$out/bench_$v.json').read().strip().splitlines()[-1])
print('c3 $v', d['ms_per_step'], round(d['roofline']['avg_launch_ms'], 4), round(d['roofline']['isolated']['avg_launch_ms'], 4))"
done
for v in A F G; do
  cp tools/ab/lib_$v.so $L
  timeout -k 10 300 python -u bench.py --config C5 --precision mixed --no-cpu-baseline --no-exact-compare > $out/c5_$v.json 2> $out/c5_$v.err; step $? c5_$v
  python3 -c "
import json; d = json.loads(open('$out/c5_$v.json').read().strip().splitlines()[-1])
print('c5 $v', d['ms_per_step'], d.get('ms_per_force_eval'), round(d['roofline']['isolated']['avg_launch_ms'], 4))"
done
cp tools/ab/lib_F.so $L
timeout -k 10 600 python -u -m pytest tests/test_gpu_cluster.py tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_mixed.py -x -v --timeout 300 --timeout-method thread > $out/tests_F.log 2>&1; step $? tests_F
grep -E "passed|failed" $out/tests_F.log | tail -2

#!/bin/bash
# round 5, session aj: same-box A/B of the k_pairs_cq variants (r05ai measured VALU -5.4 % but
# 161 -> 167 us isolated on another box, C5 2.58 -> 2.66 ms): A = ba119e2 (r05ah), B = r05ai
# (packed-byte all_ge + ballot fixed-range flag), C = B + degree-10 exp polynomial, D = A + the
# ballot flag only, E = A + the exp polynomial only.  Libraries prebuilt under tools/ab/, copied
# over the in-tree library before each run (each run is a new process).  Expected: B/D within
# +-1 % of A if the r05ai box was slow; C/E -2..-3 us on the pair kernel (2 FMAs per pair).
out=gpurun_out/r5aj
mkdir -p $out
L=openmm-chargeflux_amd/libchargeflux_hip.so
cp $L $out/lib_orig.so
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
ARGS="--steps 40 --no-cpu-baseline --no-exact-compare"
for v in A B C D E A B C D E; do
  cp tools/ab/lib_$v.so $L
  timeout -k 10 100 python -u bench.py $ARGS > $out/bench_$v.json 2> $out/bench_$v.err; step $? bench_$v
  python3 -c "
import json; d = json.loads(open('$out/bench_$v.json').read().strip().splitlines()[-1])
print('c3 $v', d['ms_per_step'], round(d['roofline']['avg_launch_ms'], 4), round(d['roofline']['isolated']['avg_launch_ms'], 4))"
done
for v in A B C D E; do
  cp tools/ab/lib_$v.so $L
  timeout -k 10 300 python -u bench.py --config C5 --precision mixed --no-cpu-baseline --no-exact-compare > $out/c5_$v.json 2> $out/c5_$v.err; step $? c5_$v
  python3 -c "
import json; d = json.loads(open('$out/c5_$v.json').read().strip().splitlines()[-1])
print('c5 $v', d['ms_per_step'], d.get('ms_per_force_eval'), round(d['roofline']['isolated']['avg_launch_ms'], 4))"
done
cp tools/ab/lib_C.so $L
timeout -k 10 600 python -u -m pytest tests/test_gpu_cluster.py tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_mixed.py -x -v --timeout 300 --timeout-method thread > $out/tests_C.log 2>&1; step $? tests_C
grep -E "passed|failed" $out/tests_C.log | tail -2

#!/bin/bash
# round 5, session aq: k_g_coeffs block sum by wave butterflies + one barrier (was an 8-round LDS
# tree per block), as k_assemble_energy in r05al.  A = HEAD library, H = the change (prebuilt under
# tools/ab/, swapped per run).  Expected: the coefficients phase 6.5 -> ~5 us, C3 step -1..-2 us (on
# the exposed tail).  Then the GPU tests that check energies, on H.
out=gpurun_out/r5aq
mkdir -p $out
L=openmm-chargeflux_amd/libchargeflux_hip.so
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
ARGS="--steps 40 --no-cpu-baseline --no-exact-compare"
for v in A H A H A H; do
  cp tools/ab/lib_$v.so $L
  timeout -k 10 100 python -u bench.py $ARGS > $out/bench_$v.json 2> $out/bench_$v.err; step $? bench_$v
  python3 -c "
import json; d = json.loads(open('$out/bench_$v.json').read().strip().splitlines()[-1])
print('c3 $v', d['ms_per_step'], d['kernels_ms_per_step']['kspace_coeffs'], round(d['roofline']['isolated']['avg_launch_ms'], 4))"
done
cp tools/ab/lib_H.so $L
timeout -k 10 700 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_overlap.py tests/test_gpu_graph.py tests/test_gpu_grid.py -x -v --timeout 300 --timeout-method thread > $out/tests_H.log 2>&1; step $? tests_H
grep -E "passed|failed" $out/tests_H.log | tail -2

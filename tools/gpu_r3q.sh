#!/bin/bash
# GPU session (round 3): same-box A/B of two grid-kernel changes -- interpolation row 0 as
# products (no zero fill) and spread source entries carrying their tile offsets (no bin-table
# read per staged piece) -- against the previous grid kernels (tmp_ab/libchargeflux_hip_base.so):
# bitwise A/B, grid tests, isolated kernel times, C3 and C5 bench alternated.  Each GPU step
# time-limited.
out=gpurun_out/r3q
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
L=openmm-chargeflux_amd/libchargeflux_hip.so
cp $L tmp_ab/libchargeflux_hip_new.so
use() { cp tmp_ab/libchargeflux_hip_$1.so $L; }
timeout -k 10 300 python -u tools/ab_bits.py run tmp_ab/libchargeflux_hip_base.so $out/ab0.npz > $out/ab0.log 2>&1; step $? ab0
timeout -k 10 300 python -u tools/ab_bits.py run tmp_ab/libchargeflux_hip_new.so $out/ab1.npz > $out/ab1.log 2>&1; step $? ab1
python tools/ab_bits.py cmp $out/ab0.npz $out/ab1.npz > $out/ab.txt 2>&1; echo "ab cmp rc=$?"; cat $out/ab.txt | tail -7
rm -f $out/ab0.npz $out/ab1.npz
timeout -k 10 300 python -u -m pytest tests/test_gpu_grid.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1; rc=$?; tail -2 $out/tests.log; step $rc tests
R=$GRAFT_REPO_ROOT
ARGS="--steps 10 --warmup 3 --no-cpu-baseline --no-exact-compare"
for v in new base; do
    use $v
    (cd /tmp && export TMPDIR=/tmp && CF_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$out/tr_$v -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/$out/tr_$v.log 2>&1); step $? tr_$v
done
for v in new base; do echo "== $v"; python3 tools/prof_stats.py $out/tr_$v/run_kernel_stats.csv 4; done
for n in new1 base1 new2 base2; do
    use ${n%?}
    timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-exact-compare > $out/bench_$n.json 2> $out/bench_$n.err; step $? bench_$n
done
for v in new base; do
    use $v
    timeout -k 10 600 python -u bench.py --config C5 --precision mixed --steps 10 --warmup 3 --no-cpu-baseline --no-exact-compare > $out/c5_$v.json 2> $out/c5_$v.err; step $? c5_$v
done
use new
python - <<'P'
import json
for n in ("new1", "base1", "new2", "base2", "c5_new", "c5_base"):
    f = f"gpurun_out/r3q/bench_{n}.json" if not n.startswith("c5") else f"gpurun_out/r3q/{n}.json"
    d = json.loads(open(f).read().strip().splitlines()[-1])
    k = d["kernels_ms_per_step"]
    print(n, d["ms_per_step"], d["ms_per_force_eval"], k["grid_spread"], k["grid_interp"])
P
exit 0

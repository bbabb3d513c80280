#!/bin/bash
# GPU session (round 3): k_excl with 4 lanes per atom for the half-list window sums (this tree)
# against the previous one-lane form (tmp_ab/libchargeflux_hip_base.so): bitwise A/B, full GPU
# test suite on the new library, isolated kernel times, C3 bench alternated.  Each GPU step
# time-limited.
out=gpurun_out/r3s
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
L=openmm-chargeflux_amd/libchargeflux_hip.so
cp $L tmp_ab/libchargeflux_hip_new.so
use() { cp tmp_ab/libchargeflux_hip_$1.so $L; }
timeout -k 10 300 python -u tools/ab_bits.py run tmp_ab/libchargeflux_hip_base.so $out/ab0.npz > $out/ab0.log 2>&1; step $? ab0
timeout -k 10 300 python -u tools/ab_bits.py run tmp_ab/libchargeflux_hip_new.so $out/ab1.npz > $out/ab1.log 2>&1; step $? ab1
python tools/ab_bits.py cmp $out/ab0.npz $out/ab1.npz > $out/ab.txt 2>&1; echo "ab cmp rc=$?"; tail -1 $out/ab.txt
rm -f $out/*.npz
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1
rc=$?; tail -2 $out/tests.log; step $rc tests
R=$GRAFT_REPO_ROOT
ARGS="--steps 10 --warmup 3 --no-cpu-baseline --no-exact-compare"
for v in new base; do
    use $v
    (cd /tmp && export TMPDIR=/tmp && CF_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$out/tr_$v -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/$out/tr_$v.log 2>&1); step $? tr_$v
done
python3 - <<'P'
import csv
for v in ("new", "base"):
    rows = list(csv.DictReader(open(f"gpurun_out/r3s/tr_{v}/run_kernel_stats.csv")))
    print(v, {r["Name"].split("(")[0]: round(float(r["AverageNs"]) / 1000, 1) for r in rows if "k_excl" in r["Name"] or "pairs_half" in r["Name"]})
P
for n in new1 base1 new2 base2; do
    use ${n%?}
    timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-exact-compare > $out/bench_$n.json 2> $out/bench_$n.err; step $? bench_$n
done
use new
python - <<'P'
import json
for n in ("new1", "base1", "new2", "base2"):
    d = json.loads(open(f"gpurun_out/r3s/bench_{n}.json").read().strip().splitlines()[-1])
    k = d["kernels_ms_per_step"]
    print(n, d["ms_per_step"], d["ms_per_force_eval"], k["direct_excl"])
P
exit 0

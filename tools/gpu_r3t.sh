#!/bin/bash
# GPU session (round 3): k_assemble_energy with 4 lanes per x-atom for the chain-rule gather
# (this tree) against one lane per atom (tmp_ab/libchargeflux_hip_base.so): A/B of outputs (the
# chain-rule sum order changes: not bitwise), full GPU test suite, isolated kernel times, C3
# bench alternated.  Each GPU step time-limited.
out=gpurun_out/r3t
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
L=openmm-chargeflux_amd/libchargeflux_hip.so
cp $L tmp_ab/libchargeflux_hip_new.so
use() { cp tmp_ab/libchargeflux_hip_$1.so $L; }
timeout -k 10 300 python -u tools/ab_bits.py run tmp_ab/libchargeflux_hip_base.so $out/ab0.npz > $out/ab0.log 2>&1; step $? ab0
timeout -k 10 300 python -u tools/ab_bits.py run tmp_ab/libchargeflux_hip_new.so $out/ab1.npz > $out/ab1.log 2>&1; step $? ab1
python tools/ab_bits.py cmp $out/ab0.npz $out/ab1.npz > $out/ab.txt 2>&1; echo "ab cmp rc=$?"; tail -3 $out/ab.txt
python - <<'P'
import numpy as np
a = np.load("gpurun_out/r3t/ab0.npz"); b = np.load("gpurun_out/r3t/ab1.npz")
worst = 0.0
for k in a.files:
    x, y = a[k].astype(float), b[k].astype(float)
    if not x.size:
        continue
    s = float(np.abs(x).max()) or 1.0
    worst = max(worst, float(np.abs(x - y).max()) / s)
print("max relative difference over every output:", worst)
P
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
    rows = list(csv.DictReader(open(f"gpurun_out/r3t/tr_{v}/run_kernel_stats.csv")))
    print(v, {r["Name"].split("(")[0]: round(float(r["AverageNs"]) / 1000, 1) for r in rows if "assemble" in r["Name"]})
P
for n in new1 base1 new2 base2; do
    use ${n%?}
    timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-exact-compare > $out/bench_$n.json 2> $out/bench_$n.err; step $? bench_$n
done
use new
python - <<'P'
import json
for n in ("new1", "base1", "new2", "base2"):
    d = json.loads(open(f"gpurun_out/r3t/bench_{n}.json").read().strip().splitlines()[-1])
    print(n, d["ms_per_step"], d["ms_per_force_eval"], d["kernels_ms_per_step"]["energy"])
P
exit 0

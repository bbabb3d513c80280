#!/bin/bash
# GPU session (round 4, first): (1) the prepared unpaired-LDS patch (tmp_ab/libchargeflux_hip_unps.so:
# k_pairs_half, spread, interpolation built with no-load-store-opt) against the current library --
# bitwise A/B, isolated kernel times, C3 bench alternated; (2) grid width W = 10..14 at C3 fp64
# against the exact k-sum.  Every GPU step is time-limited; the script stops at
# the first failure.
out=gpurun_out/r4a
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
L=openmm-chargeflux_amd/libchargeflux_hip.so
use() { cp tmp_ab/libchargeflux_hip_$1.so $L; }
timeout -k 10 300 python -u tools/ab_bits.py run tmp_ab/libchargeflux_hip_cur.so $out/ab0.npz > $out/ab0.log 2>&1; step $? ab0
timeout -k 10 300 python -u tools/ab_bits.py run tmp_ab/libchargeflux_hip_unps.so $out/ab1.npz > $out/ab1.log 2>&1; step $? ab1
python tools/ab_bits.py cmp $out/ab0.npz $out/ab1.npz > $out/ab.txt 2>&1; echo "ab cmp rc=$?"; tail -1 $out/ab.txt
rm -f $out/*.npz
R=$GRAFT_REPO_ROOT
ARGS="--steps 10 --warmup 3 --no-cpu-baseline --no-exact-compare"
for v in unps cur; do
    use $v
    (cd /tmp && export TMPDIR=/tmp && CF_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$out/tr_$v -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/$out/tr_$v.log 2>&1); step $? tr_$v
done
for n in unps1 cur1 unps2 cur2; do
    use ${n%?}
    timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-exact-compare > $out/bench_$n.json 2> $out/bench_$n.err; step $? bench_$n
done
use cur
for W in 10 11 12 13 14; do
    timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --grid-width $W > $out/w$W.json 2> $out/w$W.err; step $? w$W
done
python3 - <<'P'
import csv, json
for v in ("unps", "cur"):
    rows = list(csv.DictReader(open(f"gpurun_out/r4a/tr_{v}/run_kernel_stats.csv")))
    print(v, {r["Name"].split("(")[0][-28:]: round(float(r["AverageNs"]) / 1000, 1) for r in rows if "pairs_half" in r["Name"] or "interp" in r["Name"] or "spread" in r["Name"]})
for n in ("unps1", "cur1", "unps2", "cur2"):
    d = json.loads(open(f"gpurun_out/r4a/bench_{n}.json").read().strip().splitlines()[-1])
    print(n, d["ms_per_step"], d["ms_per_force_eval"])
for W in (10, 11, 12, 13, 14):
    d = json.loads(open(f"gpurun_out/r4a/w{W}.json").read().strip().splitlines()[-1])
    print("W", W, d["ms_per_step"], d["ms_per_force_eval"], d.get("exact_kspace"))
P
exit 0

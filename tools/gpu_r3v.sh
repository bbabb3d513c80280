#!/bin/bash
# GPU session (round 3): 8-B LDS reads left unpaired (ds_read_b64 instead of ds_read2_b64) in
# k_pairs_half, k_g_interp2 and k_g_interp4 (tmp_ab/libchargeflux_hip_unp.so; unps: also the
# spread) against the current library: bitwise A/B, isolated kernel times, C3 and C5 bench alternated.  Each GPU
# step time-limited.
out=gpurun_out/r3v
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
L=openmm-chargeflux_amd/libchargeflux_hip.so
cp $L tmp_ab/libchargeflux_hip_cur.so
use() { cp tmp_ab/libchargeflux_hip_$1.so $L; }
timeout -k 10 300 python -u tools/ab_bits.py run tmp_ab/libchargeflux_hip_cur.so $out/ab0.npz > $out/ab0.log 2>&1; step $? ab0
timeout -k 10 300 python -u tools/ab_bits.py run tmp_ab/libchargeflux_hip_unp.so $out/ab1.npz > $out/ab1.log 2>&1; step $? ab1
python tools/ab_bits.py cmp $out/ab0.npz $out/ab1.npz > $out/ab.txt 2>&1; echo "ab cmp rc=$?"; tail -1 $out/ab.txt
timeout -k 10 300 python -u tools/ab_bits.py run tmp_ab/libchargeflux_hip_unps.so $out/ab2.npz > $out/ab2.log 2>&1; step $? ab2
python tools/ab_bits.py cmp $out/ab0.npz $out/ab2.npz > $out/ab_s.txt 2>&1; echo "ab cmp unps rc=$?"; tail -1 $out/ab_s.txt
rm -f $out/*.npz
R=$GRAFT_REPO_ROOT
ARGS="--steps 10 --warmup 3 --no-cpu-baseline --no-exact-compare"
for v in unp unps cur; do
    use $v
    (cd /tmp && export TMPDIR=/tmp && CF_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$out/tr_$v -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/$out/tr_$v.log 2>&1); step $? tr_$v
done
python3 - <<'P'
import csv
for v in ("unp", "unps", "cur"):
    rows = list(csv.DictReader(open(f"gpurun_out/r3v/tr_{v}/run_kernel_stats.csv")))
    print(v, {r["Name"].split("(")[0][-28:]: round(float(r["AverageNs"]) / 1000, 1) for r in rows if "pairs_half" in r["Name"] or "interp" in r["Name"] or "spread" in r["Name"]})
P
for n in unps1 cur1 unps2 cur2 unp1; do
    use ${n%?}
    timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-exact-compare > $out/bench_$n.json 2> $out/bench_$n.err; step $? bench_$n
done
for v in unps cur; do
    use $v
    timeout -k 10 600 python -u bench.py --config C5 --precision mixed --steps 10 --warmup 3 --no-cpu-baseline --no-exact-compare > $out/c5_$v.json 2> $out/c5_$v.err; step $? c5_$v
done
use cur
python - <<'P'
import json
for n in ("unps1", "cur1", "unps2", "cur2", "unp1", "c5_unps", "c5_cur"):
    f = f"gpurun_out/r3v/bench_{n}.json" if not n.startswith("c5") else f"gpurun_out/r3v/{n}.json"
    d = json.loads(open(f).read().strip().splitlines()[-1])
    k = d["kernels_ms_per_step"]
    print(n, d["ms_per_step"], d["ms_per_force_eval"], k["direct_pairs"], k["grid_interp"], k["grid_spread"])
P
exit 0

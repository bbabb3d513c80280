#!/bin/bash
# GPU session (round 3): build-time variants against the current library (cur): tap rows
# assembled 16 / 24 atoms at a time (ot16, ot24; now 8) and the list builder capped at 128 VGPRs
# (nl4: 4 waves per SIMD, with spills).  Bitwise A/B, isolated kernel times, C3 bench.  Each GPU
# step time-limited.
out=gpurun_out/r3r
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
L=openmm-chargeflux_amd/libchargeflux_hip.so
cp $L tmp_ab/libchargeflux_hip_cur.so
use() { cp tmp_ab/libchargeflux_hip_$1.so $L; }
timeout -k 10 300 python -u tools/ab_bits.py run tmp_ab/libchargeflux_hip_cur.so $out/ab_cur.npz > $out/ab_cur.log 2>&1; step $? ab_cur
for v in ot16 ot24 nl4; do
    timeout -k 10 300 python -u tools/ab_bits.py run tmp_ab/libchargeflux_hip_$v.so $out/ab_$v.npz > $out/ab_$v.log 2>&1; step $? ab_$v
    python tools/ab_bits.py cmp $out/ab_cur.npz $out/ab_$v.npz > $out/ab_$v.txt 2>&1; echo "ab $v rc=$?"; tail -1 $out/ab_$v.txt
done
rm -f $out/*.npz
R=$GRAFT_REPO_ROOT
ARGS="--steps 10 --warmup 3 --no-cpu-baseline --no-exact-compare"
for v in cur ot16 ot24 nl4; do
    use $v
    (cd /tmp && export TMPDIR=/tmp && CF_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$out/tr_$v -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/$out/tr_$v.log 2>&1); step $? tr_$v
done
python3 - <<'P'
import csv
for v in ("cur", "ot16", "ot24", "nl4"):
    rows = list(csv.DictReader(open(f"gpurun_out/r3r/tr_{v}/run_kernel_stats.csv")))
    d = {r["Name"]: float(r["AverageNs"]) / 1000 for r in rows}
    pick = {k: round(t, 1) for k, t in d.items() if "order_taps" in k or "nlist_wave" in k}
    print(v, pick)
P
for n in cur1 ot161 nl41 cur2 ot162 nl42; do
    use ${n%?}
    timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-exact-compare > $out/bench_$n.json 2> $out/bench_$n.err; step $? bench_$n
done
use cur
python - <<'P'
import json
for n in ("cur1", "ot161", "nl41", "cur2", "ot162", "nl42"):
    d = json.loads(open(f"gpurun_out/r3r/bench_{n}.json").read().strip().splitlines()[-1])
    k = d["kernels_ms_per_step"]
    print(n, d["ms_per_step"], d["ms_per_force_eval"], k["grid_sort"], k["neighbor_list"])
P
exit 0

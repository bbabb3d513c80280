#!/bin/bash
# round 4: k_g_spread_mfma ablation -- base (kP = 32), kP = 64 (CF_SPREAD_PASS=64), spabl1 (no
# MFMAs), spabl2 (no tap loads); k_g_interp2 inabl1 (halo staging only), inabl2 (no halo loads):
# isolated kernel time at C3, fixed positions, one stream.
out=gpurun_out/r4k
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
L=openmm-chargeflux_amd/libchargeflux_hip.so
cp $L tmp_ab/libchargeflux_hip_intree.so || exit 3
R=$GRAFT_REPO_ROOT
for v in spbase p64 spabl1 spabl2 inabl1 inabl2; do
    if [ $v = p64 ]; then cp tmp_ab/libchargeflux_hip_spbase.so $L || exit 3; export CF_SPREAD_PASS=64; else cp tmp_ab/libchargeflux_hip_$v.so $L || exit 3; unset CF_SPREAD_PASS; fi
    (cd /tmp && export TMPDIR=/tmp && CF_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$out/tr_$v -o run --output-format csv -- python3 $R/tools/pair_ablation.py --evals 20 > $R/$out/tr_$v.log 2>&1); step $? tr_$v
done
unset CF_SPREAD_PASS
cp tmp_ab/libchargeflux_hip_intree.so $L
python3 - <<'P'
import csv
for v in ("spbase", "p64", "spabl1", "spabl2", "inabl1", "inabl2"):
    rows = list(csv.DictReader(open(f"gpurun_out/r4k/tr_{v}/run_kernel_stats.csv")))
    print(v, {r["Name"].split("(")[0][-24:]: (r["Calls"], round(float(r["AverageNs"]) / 1000, 1)) for r in rows if "spread" in r["Name"] or "interp" in r["Name"]})
P
timeout -k 10 500 python -u tools/scaling_probe.py --config C5 --precision mixed --worlds 1 2 4 8 --steps 20 > $out/c5_probe.jsonl 2> $out/c5_probe.err; step $? c5_probe
timeout -k 10 500 python -u tools/scaling_probe.py --config C5 --precision mixed --worlds 1 8 --steps 20 --no-timing > $out/c5_probe_wall.jsonl 2> $out/c5_probe_wall.err; step $? c5_probe_wall
cut -c1-300 $out/c5_probe_wall.jsonl

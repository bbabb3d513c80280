#!/bin/bash
# round 4: wave-decoupled k_g_spread_mfma ablation (spabl1: no MFMAs, spabl3: source lists only)
# at C3, plus the grid parity tests with the in-tree library.
out=gpurun_out/r4m
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
L=openmm-chargeflux_amd/libchargeflux_hip.so
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_grid.py -x -q --timeout 150 --timeout-method thread > $out/tests.log 2>&1; rc=$?; tail -3 $out/tests.log; step $rc tests
cp $L tmp_ab/libchargeflux_hip_intree.so || exit 3
for v in spbase spabl1 spabl3; do
    cp tmp_ab/libchargeflux_hip_$v.so $L || exit 3
    (cd /tmp && export TMPDIR=/tmp && CF_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$out/tr_$v -o run --output-format csv -- python3 $R/tools/pair_ablation.py --evals 20 > $R/$out/tr_$v.log 2>&1); step $? tr_$v
done
cp tmp_ab/libchargeflux_hip_intree.so $L
python3 - <<'P'
import csv
for v in ("spbase", "spabl1", "spabl3"):
    rows = list(csv.DictReader(open(f"gpurun_out/r4m/tr_{v}/run_kernel_stats.csv")))
    print(v, {r["Name"].split("(")[0][-24:]: (r["Calls"], round(float(r["AverageNs"]) / 1000, 1)) for r in rows if "spread" in r["Name"]})
P

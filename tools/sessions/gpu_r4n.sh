#!/bin/bash
# round 4: k_g_spread_mfma with one LDS buffer per wave (sb1, in-tree) against the same with a
# 5-waves-per-SIMD VGPR cap (wpe5): grid parity tests, isolated C3 kernel times.
out=gpurun_out/r4n
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
L=openmm-chargeflux_amd/libchargeflux_hip.so
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_grid.py -x -q --timeout 150 --timeout-method thread > $out/tests.log 2>&1; rc=$?; tail -3 $out/tests.log; step $rc tests
cp $L tmp_ab/libchargeflux_hip_intree.so || exit 3
for v in sb1 wpe5 sb1b wpe5b; do
    cp tmp_ab/libchargeflux_hip_${v%b}.so $L || exit 3
    (cd /tmp && export TMPDIR=/tmp && CF_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$out/tr_$v -o run --output-format csv -- python3 $R/tools/pair_ablation.py --evals 20 > $R/$out/tr_$v.log 2>&1); step $? tr_$v
done
cp tmp_ab/libchargeflux_hip_intree.so $L
python3 - <<'P'
import csv
for v in ("sb1", "wpe5", "sb1b", "wpe5b"):
    rows = list(csv.DictReader(open(f"gpurun_out/r4n/tr_{v}/run_kernel_stats.csv")))
    print(v, {r["Name"].split("(")[0][-24:]: (r["Calls"], round(float(r["AverageNs"]) / 1000, 1)) for r in rows if "spread" in r["Name"] or "interp" in r["Name"]})
P

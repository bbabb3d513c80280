#!/bin/bash
# round 4: k_pairs_cq ablation (abl1: no pair term; abl2: no partner-side LDS atomics) against the
# full kernel (w16) and the per-atom list (CF_CLUSTER=0), fixed positions, one stream.
out=gpurun_out/r4g
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
L=openmm-chargeflux_amd/libchargeflux_hip.so
cp $L tmp_ab/libchargeflux_hip_intree.so || exit 3
R=$GRAFT_REPO_ROOT
for v in w16 abl1 abl2 atom; do
    if [ $v = atom ]; then cp tmp_ab/libchargeflux_hip_w16.so $L || exit 3; export CF_CLUSTER=0; else cp tmp_ab/libchargeflux_hip_$v.so $L || exit 3; unset CF_CLUSTER; fi
    (cd /tmp && export TMPDIR=/tmp && CF_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$out/tr_$v -o run --output-format csv -- python3 $R/tools/pair_ablation.py --evals 20 > $R/$out/tr_$v.log 2>&1); step $? tr_$v
done
unset CF_CLUSTER
cp tmp_ab/libchargeflux_hip_intree.so $L
python3 - <<'P'
import csv
for v in ("w16", "abl1", "abl2", "atom"):
    rows = list(csv.DictReader(open(f"gpurun_out/r4g/tr_{v}/run_kernel_stats.csv")))
    print(v, {r["Name"].split("(")[0][-26:]: (r["Calls"], round(float(r["AverageNs"]) / 1000, 1)) for r in rows if "pairs" in r["Name"] or "cl_build" in r["Name"] or "nlist" in r["Name"] or "k_excl" in r["Name"]})
P

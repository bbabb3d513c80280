#!/bin/bash
# round 4: k_pairs_cq variants A/B (base = committed; w16 = packed tests + phase-B prefetch;
# w12 = the same at 12 waves per block, 168 VGPRs): bitwise A/B, isolated kernel time, C3 bench.
out=gpurun_out/r4f
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
L=openmm-chargeflux_amd/libchargeflux_hip.so
cp $L tmp_ab/libchargeflux_hip_intree.so || exit 3
use() { cp tmp_ab/libchargeflux_hip_$1.so $L || exit 3; }
for v in w16 w12; do
    use $v
    timeout -k 10 300 python -u -m pytest tests/test_gpu_cluster.py -x -q --timeout 150 --timeout-method thread > $out/tests_$v.log 2>&1; rc=$?; tail -1 $out/tests_$v.log; step $rc tests_$v
done
R=$GRAFT_REPO_ROOT
for v in base w16 w12; do
    use $v
    (cd /tmp && export TMPDIR=/tmp && CF_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$out/tr_$v -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-exact-compare > $R/$out/tr_$v.log 2>&1); step $? tr_$v
done
for n in base1 w161 w121 base2 w162 w122; do
    use ${n%?}
    timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-exact-compare > $out/bench_$n.json 2> $out/bench_$n.err; step $? bench_$n
done
cp tmp_ab/libchargeflux_hip_intree.so $L
python3 - <<'P'
import csv, json
for v in ("base", "w16", "w12"):
    rows = list(csv.DictReader(open(f"gpurun_out/r4f/tr_{v}/run_kernel_stats.csv")))
    print(v, {r["Name"].split("(")[0][-30:]: round(float(r["AverageNs"]) / 1000, 1) for r in rows if "pairs_cq" in r["Name"] or "cl_build" in r["Name"]})
for n in ("base1", "w161", "w121", "base2", "w162", "w122"):
    d = json.loads(open(f"gpurun_out/r4f/bench_{n}.json").read().strip().splitlines()[-1])
    print(n, d["ms_per_step"], d["ms_per_force_eval"], d["kernels_ms_per_step"]["direct_pairs"])
P

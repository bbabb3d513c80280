#!/bin/bash
# round 4: cluster-pair list vs the per-atom half list (CF_CLUSTER=0) -- parity, isolated kernel
# trace of both, C3 bench alternated.
out=gpurun_out/r4d
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_cluster.py tests/test_gpu_half.py -x -q --timeout 150 --timeout-method thread > $out/tests.log 2>&1; rc=$?; tail -2 $out/tests.log; step $rc tests
R=$GRAFT_REPO_ROOT
for v in cq half; do
    if [ $v = half ]; then export CF_CLUSTER=0; else unset CF_CLUSTER; fi
    (cd /tmp && export TMPDIR=/tmp && CF_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$out/tr_$v -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-exact-compare > $R/$out/tr_$v.log 2>&1); step $? tr_$v
done
for n in cq1 half1 cq2 half2; do
    if [ ${n%?} = half ]; then export CF_CLUSTER=0; else unset CF_CLUSTER; fi
    timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-exact-compare > $out/bench_$n.json 2> $out/bench_$n.err; step $? bench_$n
done
unset CF_CLUSTER
python3 - <<'P'
import csv, json
for v in ("cq", "half"):
    rows = list(csv.DictReader(open(f"gpurun_out/r4d/tr_{v}/run_kernel_stats.csv")))
    tot = sum(float(r["TotalDurationNs"]) for r in rows) / 1e3 / 13
    print(v, "kernel-us/step", round(tot, 1), {r["Name"].split("(")[0][-24:]: round(float(r["TotalDurationNs"]) / 1e3 / 13, 1) for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:9]})
for n in ("cq1", "half1", "cq2", "half2"):
    d = json.loads(open(f"gpurun_out/r4d/bench_{n}.json").read().strip().splitlines()[-1])
    k = d["kernels_ms_per_step"]
    print(n, d["ms_per_step"], d["ms_per_force_eval"], "pairs", k["direct_pairs"], "list", k["neighbor_list"], "cells", k["cell_sort"])
P

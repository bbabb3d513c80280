#!/bin/bash
# round 4: k_pairs_cq phase A with the listed-pair and range ballots ANDed on the scalar unit
# (bit-identical): cluster / half tests, isolated C3 kernel time, C3 bench x2.
out=gpurun_out/r4v
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_cluster.py tests/test_gpu_half.py -x -q --timeout 150 --timeout-method thread > $out/tests.log 2>&1; rc=$?; tail -2 $out/tests.log; step $rc tests
(cd /tmp && export TMPDIR=/tmp && CF_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$out/tr -o run --output-format csv -- python3 $R/tools/pair_ablation.py --evals 20 > $R/$out/tr.log 2>&1); step $? tr
python3 - <<'P'
import csv
rows = list(csv.DictReader(open("gpurun_out/r4v/tr/run_kernel_stats.csv")))
print({r["Name"].split("(")[0][-24:]: (r["Calls"], round(float(r["AverageNs"]) / 1000, 1)) for r in rows if "pairs" in r["Name"] or "interp" in r["Name"] or "spread" in r["Name"]})
P
for n in 1 2; do
    timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-exact-compare > $out/bench_$n.json 2> $out/bench_$n.err; step $? bench_$n
    python3 -c "import json; d = json.loads(open('$out/bench_$n.json').read().strip().splitlines()[-1]); print('bench', d['ms_per_step'], d['kernels_ms_per_step']['direct_pairs'])"
done

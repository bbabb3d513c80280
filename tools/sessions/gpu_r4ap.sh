#!/bin/bash
# round 4: k_assemble_energy with several 256-atom chunks per block at large N (as k_g_bin, r4ao):
# full GPU suite, C5 isolated at CF_BIN_ROUNDS = 1 / default on one box, C5 and C3 benches.
out=gpurun_out/r4ap
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1; rc=$?; tail -2 $out/tests.log; step $rc tests
for r in 1 0; do
    (cd /tmp && export TMPDIR=/tmp && CF_BIN_ROUNDS=$r CF_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$out/tr_$r -o run --output-format csv -- python3 $R/tools/pair_ablation.py --config C5 --precision mixed --evals 6 > $R/$out/tr_$r.log 2>&1); step $? tr_$r
    python3 - $r <<'P'
import csv, sys
rows = list(csv.DictReader(open(f"gpurun_out/r4ap/tr_{sys.argv[1]}/run_kernel_stats.csv")))
print("rounds", sys.argv[1], {r["Name"].split("(")[0][-18:]: (r["Calls"], round(float(r["AverageNs"]) / 1000, 1)) for r in rows if "k_g_bin" in r["Name"] or "assemble" in r["Name"]})
P
done
timeout -k 10 400 python -u bench.py --config C5 --precision mixed --steps 10 --warmup 3 --no-cpu-baseline --no-exact-compare > $out/c5.json 2> $out/c5.err; step $? c5
python3 -c "import json; d = json.loads(open('$out/c5.json').read().strip().splitlines()[-1]); print('c5', d['ms_per_step'])"
timeout -k 10 300 python -u bench.py > $out/c3.json 2> $out/c3.err; step $? c3
python3 -c "import json; d = json.loads(open('$out/c3.json').read().strip().splitlines()[-1]); print('c3', d['ms_per_step'], d['value'])"

#!/bin/bash
# round 4: 16-B halo staging in the two- and four-atom interpolation: grid tests, isolated C3 and
# C5 kernel times, C3 bench.
out=gpurun_out/r4t
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_grid.py tests/test_gpu_mixed.py -x -q --timeout 150 --timeout-method thread > $out/tests.log 2>&1; rc=$?; tail -2 $out/tests.log; step $rc tests
(cd /tmp && export TMPDIR=/tmp && CF_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$out/tr_c3 -o run --output-format csv -- python3 $R/tools/pair_ablation.py --evals 20 > $R/$out/tr_c3.log 2>&1); step $? tr_c3
(cd /tmp && export TMPDIR=/tmp && CF_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$out/tr_c5 -o run --output-format csv -- python3 $R/tools/pair_ablation.py --config C5 --precision mixed --evals 6 > $R/$out/tr_c5.log 2>&1); step $? tr_c5
python3 - <<'P'
import csv
for v in ("tr_c3", "tr_c5"):
    rows = list(csv.DictReader(open(f"gpurun_out/r4t/{v}/run_kernel_stats.csv")))
    print(v, {r["Name"].split("(")[0][-24:]: (r["Calls"], round(float(r["AverageNs"]) / 1000, 1)) for r in rows if "k_g_" in r["Name"] or "pairs" in r["Name"]})
P
timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-exact-compare > $out/bench.json 2> $out/bench.err; step $? bench
python3 -c "import json; d = json.loads(open('$out/bench.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d.get('graph_replay_ms_per_step'), d['kernels_ms_per_step']['grid_interp'])"

#!/bin/bash
# round 4: tap rows store (W + 8) / 2 of the 12 pairs per row at every width (11 at W = 14): grid +
# mixed tests, C3 isolated k_g_order_taps<14> (was ~23 us), C3 benches.
out=gpurun_out/r4am
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_grid.py tests/test_gpu_mixed.py -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1; rc=$?; tail -2 $out/tests.log; step $rc tests
(cd /tmp && export TMPDIR=/tmp && CF_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$out/tr -o run --output-format csv -- python3 $R/tools/pair_ablation.py --evals 20 > $R/$out/tr.log 2>&1); step $? tr
python3 - <<'P'
import csv
rows = list(csv.DictReader(open("gpurun_out/r4am/tr/run_kernel_stats.csv")))
print({r["Name"].split("(")[0][-24:]: (r["Calls"], round(float(r["AverageNs"]) / 1000, 1)) for r in rows if "k_g_" in r["Name"]})
P
for n in 1 2; do
    timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-exact-compare > $out/bench_$n.json 2> $out/bench_$n.err; step $? bench_$n
    python3 -c "import json; d = json.loads(open('$out/bench_$n.json').read().strip().splitlines()[-1]); print('bench', d['ms_per_step'], d['kernels_ms_per_step'].get('grid_sort'))"
done

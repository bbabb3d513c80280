#!/bin/bash
# round 4: k_g_bin with several 256-atom rounds per block at large N (fewer increments of the one ticket
# address): grid + mixed + multi-rank tests, C5 isolated k_g_bin (was 71 us, r4ak), C5 benches (2.724-2.731).

out=gpurun_out/r4an
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_grid.py tests/test_gpu_mixed.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1; rc=$?; tail -2 $out/tests.log; step $rc tests
(cd /tmp && export TMPDIR=/tmp && CF_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$out/tr_c5 -o run --output-format csv -- python3 $R/tools/pair_ablation.py --config C5 --precision mixed --evals 6 > $R/$out/tr_c5.log 2>&1); step $? tr_c5
python3 - <<'P'
import csv
rows = list(csv.DictReader(open("gpurun_out/r4an/tr_c5/run_kernel_stats.csv")))
print({r["Name"].split("(")[0][-26:]: (r["Calls"], round(float(r["AverageNs"]) / 1000, 1)) for r in rows[:12]})
P
for n in 1 2; do
    timeout -k 10 400 python -u bench.py --config C5 --precision mixed --steps 10 --warmup 3 --no-cpu-baseline --no-exact-compare > $out/c5_$n.json 2> $out/c5_$n.err; step $? c5_$n
    python3 -c "import json; d = json.loads(open('$out/c5_$n.json').read().strip().splitlines()[-1]); print('c5', d['ms_per_step'], d['kernels_ms_per_step'].get('grid_sort'))"
done

#!/bin/bash
# round 4: k_g_spread_mfma with the 4 groups of a block unrolled (24 reads, then 16 MFMAs):
# grid tests, isolated C3 time, MFMA busy counter, C3 benches.
out=gpurun_out/r4aj
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_grid.py -x -q --timeout 150 --timeout-method thread > $out/tests.log 2>&1; rc=$?; tail -2 $out/tests.log; step $rc tests
(cd /tmp && export TMPDIR=/tmp && CF_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$out/tr -o run --output-format csv -- python3 $R/tools/pair_ablation.py --evals 20 > $R/$out/tr.log 2>&1); step $? tr
python3 - <<'P'
import csv
rows = list(csv.DictReader(open("gpurun_out/r4aj/tr/run_kernel_stats.csv")))
print({r["Name"].split("(")[0][-24:]: (r["Calls"], round(float(r["AverageNs"]) / 1000, 1)) for r in rows if "spread" in r["Name"] or "interp" in r["Name"]})
P
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_WAIT_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-include-regex "k_g_spread" -d $R/$out/pmc -o run --output-format csv -- python3 $R/bench.py --kspace-algo 2 --no-cpu-baseline --no-exact-compare --steps 3 --warmup 1 > $R/$out/pmc.log 2>&1); step $? pmc
python3 tools/pmc_show.py $out/pmc | tee $out/pmc.txt
for n in 1 2; do
    timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-exact-compare > $out/bench_$n.json 2> $out/bench_$n.err; step $? bench_$n
    python3 -c "import json; d = json.loads(open('$out/bench_$n.json').read().strip().splitlines()[-1]); print('bench', d['ms_per_step'], d['kernels_ms_per_step']['grid_spread'])"
done

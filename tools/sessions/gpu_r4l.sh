#!/bin/bash
# round 4: wave-decoupled k_g_spread_mfma -- grid parity tests, isolated kernel time at C3 and
# C5 against the vector spread, alternated C3 benches.
out=gpurun_out/${1:-r4l}
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_grid.py -x -q --timeout 150 --timeout-method thread > $out/tests.log 2>&1; rc=$?; tail -3 $out/tests.log; step $rc tests
for v in mfma vec; do
    case $v in mfma) E="";; vec) E="CF_SPREAD_MFMA=0";; esac
    (cd /tmp && export TMPDIR=/tmp && export CF_OVERLAP=0 $E && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$out/tr_$v -o run --output-format csv -- python3 $R/tools/pair_ablation.py --evals 20 > $R/$out/tr_$v.log 2>&1); step $? tr_$v
    (cd /tmp && export TMPDIR=/tmp && export CF_OVERLAP=0 $E && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$out/c5_$v -o run --output-format csv -- python3 $R/tools/pair_ablation.py --config C5 --precision mixed --evals 6 > $R/$out/c5_$v.log 2>&1); step $? c5_$v
done
for n in mfma1 vec1 mfma2 vec2; do
    case $n in mfma*) unset CF_SPREAD_MFMA;; vec*) export CF_SPREAD_MFMA=0;; esac
    timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-exact-compare > $out/bench_$n.json 2> $out/bench_$n.err; step $? bench_$n
done
unset CF_SPREAD_MFMA
export OUTN=$out
python3 - <<'P'
import csv, json, os
o = os.environ["OUTN"]
for v in ("tr_mfma", "tr_vec", "c5_mfma", "c5_vec"):
    rows = list(csv.DictReader(open(f"{o}/{v}/run_kernel_stats.csv")))
    print(v, {r["Name"].split("(")[0][-24:]: (r["Calls"], round(float(r["AverageNs"]) / 1000, 1)) for r in rows if "spread" in r["Name"] or "interp" in r["Name"]})
for n in ("mfma1", "vec1", "mfma2", "vec2"):
    d = json.loads(open(f"{o}/bench_{n}.json").read().strip().splitlines()[-1])
    print(n, d["ms_per_step"], d["ms_per_force_eval"], d["kernels_ms_per_step"]["grid_spread"])
P

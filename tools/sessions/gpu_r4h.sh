#!/bin/bash
# round 4: the matrix-core spread (k_g_spread_mfma) -- parity tests, isolated kernel time at C3
# and C5 against the vector spread (CF_SPREAD_MFMA=0) and the 128-atom pass (CF_SPREAD_PASS=128),
# alternated C3 benches, one PMC pass (VALU / MFMA / LDS / wait) over the spread kernels.
out=gpurun_out/${1:-r4h}
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_grid.py ${TESTS:-tests/test_gpu_half.py} -x -q --timeout 150 --timeout-method thread > $out/tests.log 2>&1; rc=$?; tail -3 $out/tests.log; step $rc tests
for v in mfma vec p128 p32; do
    case $v in mfma) E="";; vec) E="CF_SPREAD_MFMA=0";; p128) E="CF_SPREAD_PASS=128";; p32) E="CF_SPREAD_PASS=32";; esac
    (cd /tmp && export TMPDIR=/tmp && export CF_OVERLAP=0 $E && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$out/tr_$v -o run --output-format csv -- python3 $R/tools/pair_ablation.py --evals 20 > $R/$out/tr_$v.log 2>&1); step $? tr_$v
done
for v in mfma vec; do
    case $v in mfma) E="CF_OVERLAP=0";; vec) E="CF_SPREAD_MFMA=0 CF_OVERLAP=0";; esac
    (cd /tmp && export TMPDIR=/tmp && export $E && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$out/c5_$v -o run --output-format csv -- python3 $R/tools/pair_ablation.py --config C5 --precision mixed --evals 6 > $R/$out/c5_$v.log 2>&1); step $? c5_$v
done
for n in mfma1 vec1 mfma2 vec2; do
    case $n in mfma*) unset CF_SPREAD_MFMA;; vec*) export CF_SPREAD_MFMA=0;; esac
    timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-exact-compare > $out/bench_$n.json 2> $out/bench_$n.err; step $? bench_$n
done
unset CF_SPREAD_MFMA
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS --kernel-include-regex "k_g_spread|k_g_interp" -d $R/$out/pmc_sq -o run --output-format csv -- python3 $R/bench.py --kspace-algo 2 --no-cpu-baseline --no-exact-compare --steps 3 --warmup 1 > $R/$out/pmc_sq.log 2>&1); step $? pmc_sq
python3 tools/pmc_show.py $out/pmc_sq > $out/pmc_sq.txt
export OUTN=${1:-r4h}
python3 - <<'P'
import csv, json, os
for v in ("tr_mfma", "tr_vec", "tr_p128", "tr_p32", "c5_mfma", "c5_vec"):
    rows = list(csv.DictReader(open(f"gpurun_out/{os.environ['OUTN']}/{v}/run_kernel_stats.csv")))
    print(v, {r["Name"].split("(")[0][-24:]: (r["Calls"], round(float(r["AverageNs"]) / 1000, 1)) for r in rows if "k_g_" in r["Name"]})
for n in ("mfma1", "vec1", "mfma2", "vec2"):
    d = json.loads(open(f"gpurun_out/{os.environ['OUTN']}/bench_{n}.json").read().strip().splitlines()[-1])
    print(n, d["ms_per_step"], d["ms_per_force_eval"], d["kernels_ms_per_step"])
P
cat $out/pmc_sq.txt

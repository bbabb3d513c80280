#!/bin/bash
# GPU session (round 3): half-list pair kernel with 4-8 lanes per row over the concatenated
# sub-lists (walk_row, padded chunks) and the W <= 8 four-atom interpolation: full GPU test
# suite, isolated kernel times for CF_HALF_LPR 8 / 4, C3 bench A/B, C5 bench.  Each GPU step
# time-limited; stops at the first step that faults, aborts or times out.
out=gpurun_out/r3m
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1
rc=$?; tail -4 $out/tests.log; echo "tests rc=$rc"; [ $rc -le 1 ] || exit $rc
R=$GRAFT_REPO_ROOT
ARGS="--steps 10 --warmup 3 --no-cpu-baseline --no-exact-compare"
cd /tmp && export TMPDIR=/tmp
CF_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$out/tr8 -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/$out/tr8.log 2>&1; step $? tr8
CF_OVERLAP=0 CF_HALF_LPR=4 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$out/tr4 -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/$out/tr4.log 2>&1; step $? tr4
cd $R
echo "== isolated, lanes per row up to 8"; python3 tools/prof_stats.py $out/tr8/run_kernel_stats.csv 8
echo "== isolated, 4 lanes per row"; python3 tools/prof_stats.py $out/tr4/run_kernel_stats.csv 4
for n in a8 a4 b8; do
    env CF_HALF_LPR=${n:1} timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-exact-compare > $out/bench_$n.json 2> $out/bench_$n.err; step $? bench_$n
done
python - <<'P'
import json
for n in ("a8", "a4", "b8"):
    d = json.loads(open(f"gpurun_out/r3m/bench_{n}.json").read().strip().splitlines()[-1])
    print(n, d["ms_per_step"], d["ms_per_force_eval"], d["roofline"].get("isolated"))
P
timeout -k 10 600 python -u bench.py --config C5 --precision mixed --steps 10 --warmup 3 --no-cpu-baseline --no-exact-compare > $out/bench_c5.json 2> $out/bench_c5.err; step $? bench_c5
python - <<'P'
import json
d = json.loads(open("gpurun_out/r3m/bench_c5.json").read().strip().splitlines()[-1])
print("C5", d["ms_per_step"], d["value"], d["kernels_ms_per_step"])
P
exit 0

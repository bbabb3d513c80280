#!/bin/bash
# round 4: first GPU run of the cluster-pair half list (k_cl_build + k_pairs_cq): parity tests,
# then the C3 bench and an isolated rocprofv3 kernel trace.  Each step time-limited; stop at the
# first failure.
out=gpurun_out/r4b
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_cluster.py tests/test_gpu_half.py tests/test_gpu_graph.py tests/test_gpu_overlap.py -x -v --timeout 150 --timeout-method thread > $out/tests.log 2>&1; rc=$?; tail -25 $out/tests.log; step $rc tests
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $out/bench.json 2> $out/bench.err; step $? bench
tail -c 1500 $out/bench.json
R=$GRAFT_REPO_ROOT
(cd /tmp && export TMPDIR=/tmp && CF_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$out/tr -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-exact-compare > $R/$out/tr.log 2>&1); step $? trace
python3 - <<'P'
import csv
rows = list(csv.DictReader(open("gpurun_out/r4b/tr/run_kernel_stats.csv")))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:16]:
    print(r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1000, 1))
P

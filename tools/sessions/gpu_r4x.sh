#!/bin/bash
# round 4: phase timing events with a device-scope release (hipEventReleaseToDevice): the bench's
# event-timed dominant launch against the rocprofv3 kernel trace of the same command.
out=gpurun_out/r4x
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
R=$GRAFT_REPO_ROOT
for n in 1 2; do
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-exact-compare > $out/bench_$n.json 2> $out/bench_$n.err; step $? bench_$n
    python3 -c "import json; d = json.loads(open('$out/bench_$n.json').read().strip().splitlines()[-1]); r = d['roofline']; print('bench', d['ms_per_step'], r['avg_launch_ms'], r['frac'], r['isolated']['avg_launch_ms'], d['kernels_ms_per_step']['direct_pairs'])"
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$out/tr -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-exact-compare > $R/$out/tr.log 2>&1); step $? tr
python3 - <<'P'
import csv, json
rows = list(csv.DictReader(open("gpurun_out/r4x/tr/run_kernel_stats.csv")))
print({r["Name"].split("(")[0][-24:]: (r["Calls"], round(float(r["AverageNs"]) / 1000, 1)) for r in rows if "pairs" in r["Name"]})
d = json.loads([l for l in open("gpurun_out/r4x/tr.log") if l.startswith("{")][-1])
print("bench under trace", d["ms_per_step"], d["roofline"]["avg_launch_ms"])
P

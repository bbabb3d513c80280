#!/bin/bash
# round 4: rank-0 probe at W = 8 (C3): per-phase times and a kernel trace of the same probe.
out=gpurun_out/r4aa
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/scaling_probe.py --worlds 8 --steps 40 > $out/probe_w8_phases.jsonl 2> $out/probe.err; step $? probe
cut -c1-600 $out/probe_w8_phases.jsonl
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$out/tr -o run --output-format csv -- python3 $R/tools/scaling_probe.py --worlds 8 --steps 40 --no-timing > $R/$out/tr.log 2>&1); step $? tr
python3 - <<'P'
import csv
rows = list(csv.DictReader(open("gpurun_out/r4aa/tr/run_kernel_stats.csv")))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows[:30]:
    print(f'{r["Name"].split("(")[0][-40:]:42s} {r["Calls"]:>6s} {float(r["AverageNs"])/1000:8.1f} {float(r["TotalDurationNs"])/tot*100:6.1f}%')
P

#!/bin/bash
# GPU session (round 3): rank-0 kernel timeline at W = 8 (scaling probe under a rocprofv3 kernel
# trace), to see what the 12k-owned-atom step spends its time on.  Each GPU step time-limited.
out=gpurun_out/r3o
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/scaling_probe.py --worlds 8 --no-timing --neighbor-skin 0.15 > $out/probe8.json 2> $out/probe8.err; step $? probe8
cut -c1-200 $out/probe8.json
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$out/tr8 -o run --output-format csv -- python3 $R/tools/scaling_probe.py --worlds 8 --no-timing --neighbor-skin 0.15 > $R/$out/tr8.log 2>&1); step $? tr8
python3 tools/prof_stats.py $out/tr8/run_kernel_stats.csv 30
exit 0

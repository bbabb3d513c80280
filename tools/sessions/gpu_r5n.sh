#!/bin/bash
# round 5, session n: the multi-rank per-rank cost (rank 0 of a W-way C3 decomposition on one GPU,
# no collectives, tools/scaling_probe.py) at the current code (event hand-overs), wall time and
# per-phase GPU time, plus a kernel trace of the W = 8 rank: what a rank at N = 8 spends its
# ~0.2 ms on.  Expected: W = 8 ~0.20 ms (round 4: 0.197 with memory hand-overs).
out=gpurun_out/r5n
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
timeout -k 10 200 python -u tools/scaling_probe.py --worlds 1 2 4 8 --neighbor-skin 0.15 --no-timing > $out/probe_wall.jsonl 2> $out/probe_wall.err; step $? wall
cat $out/probe_wall.jsonl | python3 -c "import sys,json;[print(d['world'],d['ms_per_step'],d['host_enqueue_ms_per_step']) for d in map(json.loads,sys.stdin)]"
timeout -k 10 200 python -u tools/scaling_probe.py --worlds 8 --neighbor-skin 0.15 > $out/probe_phases.jsonl 2> $out/probe_phases.err; step $? phases
cat $out/probe_phases.jsonl
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/trace8 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/scaling_probe.py --worlds 8 --neighbor-skin 0.15 --no-timing --steps 20 > $GRAFT_REPO_ROOT/$out/trace8.log 2>&1); step $? trace8
python3 tools/prof_stats.py $out/trace8/run_kernel_stats.csv 30

#!/bin/bash
# round 4: rank-0 probes at the bench's skin (0.15 nm), C3, W = 1/2/4/8, no per-phase events and
# with them (phases).
out=gpurun_out/r4ab
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
timeout -k 10 400 python -u tools/scaling_probe.py --worlds 1 2 4 8 --steps 40 --neighbor-skin 0.15 --no-timing > $out/probe_wall.jsonl 2> $out/probe_wall.err; step $? probe_wall
timeout -k 10 400 python -u tools/scaling_probe.py --worlds 1 2 4 8 --steps 40 --neighbor-skin 0.15 > $out/probe_phases.jsonl 2> $out/probe_phases.err; step $? probe_phases
cut -c1-140 $out/probe_wall.jsonl

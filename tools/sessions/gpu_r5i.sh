#!/bin/bash
# round 5, session i: graph replay slows down over a run (bench graph pass: 0.5 ms/step at 5
# steps, 2.8 ms at 30, 4 s at 40 in r5c -- the r5d "hang" was that pass).  Per-20-step replay
# times for both hand-overs, and eager for comparison.
out=gpurun_out/r5i
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
timeout -k 10 60 python -u tools/graph_probe.py --graph 0 --steps 100 2>&1 | tee $out/eager.txt; step $? eager
timeout -k 10 90 python -u tools/graph_probe.py --handover memory --steps 200 2>&1 | tee $out/memory.txt; step $? memory
timeout -k 10 90 python -u tools/graph_probe.py --handover event --steps 200 2>&1 | tee $out/event.txt; step $? event

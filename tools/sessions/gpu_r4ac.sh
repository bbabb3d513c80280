#!/bin/bash
# round 4: neighbour skin at W = 8 (rank-0 probe, C3, full per-atom list): 0.15 / 0.2 / 0.25 / 0.3 nm.
out=gpurun_out/r4ac
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
for sk in 0.15 0.2 0.25 0.3; do
    timeout -k 10 300 python -u tools/scaling_probe.py --worlds 8 4 2 --steps 60 --neighbor-skin $sk --no-timing > $out/probe_$sk.jsonl 2> $out/probe_$sk.err; step $? probe_$sk
    python3 -c "
import json
for l in open('$out/probe_$sk.jsonl'):
    d = json.loads(l); print('skin $sk W', d['world'], d['ms_per_step'])"
done

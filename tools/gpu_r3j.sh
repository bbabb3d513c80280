#!/bin/bash
# GPU session (round 3): neighbour-skin sweep at the current kernels (C3 bench, 40 steps each),
# then the round's rocprofv3 evidence for the default bench command (kernel trace + stats,
# SQ / FETCH_SIZE / WRITE_SIZE passes; tools/profile_round.sh).  Each GPU step time-limited.
out=gpurun_out/r3j
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
for sk in 0.1 0.125 0.15 0.175 0.2; do
    timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-exact-compare --neighbor-skin $sk > $out/skin_$sk.json 2> $out/skin_$sk.err; step $? skin_$sk
done
python - <<'P'
import json
for sk in ("0.1", "0.125", "0.15", "0.175", "0.2"):
    d = json.loads(open(f"gpurun_out/r3j/skin_{sk}.json").read().strip().splitlines()[-1])
    k = d["kernels_ms_per_step"]
    print(sk, d["ms_per_step"], d["ms_per_force_eval"], d["config"]["nlist_builds_in_timed_steps"], k["direct_pairs"], k["neighbor_list"])
P
timeout -k 10 1000 bash tools/profile_round.sh r03j > $out/profile_round.log 2>&1; step $? profile_round
tail -12 $out/profile_round.log | cut -c1-300
exit 0

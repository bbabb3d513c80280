#!/bin/bash
# GPU session (round 3): second-stream priority A/B (CF_AUX_PRIORITY low / high / default),
# C3 bench, 40 steps each, default twice (box noise).  Each GPU step time-limited.
out=gpurun_out/r3k
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
run() {   # name, env assignment
    env $2 timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-exact-compare > $out/$1.json 2> $out/$1.err; step $? $1
}
run def1 CF_AUX_PRIORITY=
run low CF_AUX_PRIORITY=low
run high CF_AUX_PRIORITY=high
run def2 CF_AUX_PRIORITY=
python - <<'P'
import json
for n in ("def1", "low", "high", "def2"):
    d = json.loads(open(f"gpurun_out/r3k/{n}.json").read().strip().splitlines()[-1])
    print(n, d["ms_per_step"], d["ms_per_force_eval"], d["graph_replay_ms_per_step"])
P
exit 0

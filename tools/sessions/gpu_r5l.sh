#!/bin/bash
# round 5, session l: C5 (768k atoms, mixed precision) with the three one-rank lists -- the per-atom
# half list (auto), the 18-cell cluster list, the octant list.  The octant list writes 8 window
# partials per atom instead of 18 (k_excl: 119 us reading 281 MB at C5 in round 4).  Expected:
# octant k_excl ~40-60 us; pairs within 10 % of the per-atom list's 1.23 ms.
out=gpurun_out/r5l
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
ARGS="--config C5 --precision mixed --steps 20 --warmup 3 --no-cpu-baseline --no-exact-compare"
for pl in auto octant cluster; do
  timeout -k 10 200 python -u bench.py $ARGS --pair-list $pl > $out/bench_$pl.json 2> $out/bench_$pl.err; step $? $pl
done
python3 - <<'PY'
import json
for pl in ("auto", "octant", "cluster"):
    d = json.loads(open(f"gpurun_out/r5l/bench_{pl}.json").read().strip().splitlines()[-1])
    print(pl, d["ms_per_step"], d["ms_per_force_eval"], d.get("graph_replay_ms_per_step"), d["config"].get("fp64_rescan_fallbacks_in_timed_steps"),
          {k: v for k, v in d["kernels_ms_per_step"].items() if v > 0.01})
PY

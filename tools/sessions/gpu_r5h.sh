#!/bin/bash
# round 5, session h: (1) neighbour skin for the cluster-pair list (the round-2 optimum 0.15 was for
# the per-atom list; k_cl_build is 9 us per build, the phase-A slots scale with (rc + skin)^3);
# (2) the grid width W = 12 against 14: spread + interpolation ~ W^3 (0.63x), force error vs the
# exact k-sum measured at C3 (needs <= 1e-6, the grid tests' bar; W = 14: 6.5e-9); (3) repeated
# benches, each under its own limit, to see whether the r5d hang recurs.
out=gpurun_out/r5h
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
ARGS="--steps 30 --no-cpu-baseline --no-exact-compare"
for sk in 0.08 0.10 0.12 0.15 0.20; do
  timeout -k 10 100 python -u bench.py $ARGS --neighbor-skin $sk > $out/bench_skin$sk.json 2> $out/bench_skin$sk.err; step $? skin$sk
done
for w in 12 14; do
  timeout -k 10 150 python -u bench.py --steps 30 --no-cpu-baseline --grid-width $w > $out/bench_w$w.json 2> $out/bench_w$w.err; step $? w$w
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r5h/bench_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    ex = d.get("exact_kspace") or {}
    print(f.split("/")[-1], d["ms_per_step"], d.get("graph_replay_ms_per_step"), d["config"].get("nlist_builds_in_timed_steps"),
          {k: d["kernels_ms_per_step"][k] for k in ("direct_pairs", "neighbor_list", "grid_spread", "grid_interp", "grid_sort")},
          ex.get("max_abs_dforce_grid_vs_exact"), ex.get("rms_rel_dforce_vs_exact"))
PY

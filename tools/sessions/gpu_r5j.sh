#!/bin/bash
# round 5, session j: (1) the bench with its harness pass restoring the MD state (the graph pass
# ran on K steps of free flight: the r5d "hang", 4 s per step at K = 40); (2) the direct chain on
# a CU-masked second stream (cf_options.direct_cus) so that the reciprocal chain's DFT stages run
# beside the pair kernel instead of after it (r5f timeline: k_g_dft8_zfwd waited 185 us).
# Expected: graph pass ~0.45 ms/step at K = 40; direct_cus 240/224 step -10..-30 us or nothing.
out=gpurun_out/r5j
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
ARGS="--steps 40 --no-cpu-baseline --no-exact-compare"
for cu in 0 240 224 192; do
  timeout -k 10 100 python -u bench.py $ARGS --direct-cus $cu > $out/bench_cu$cu.json 2> $out/bench_cu$cu.err; step $? cu$cu
done
python3 - <<'PY'
import json, glob
for cu in (0, 240, 224, 192):
    d = json.loads(open(f"gpurun_out/r5j/bench_cu{cu}.json").read().strip().splitlines()[-1])
    print(cu, d["ms_per_step"], d.get("graph_replay_ms_per_step"), d["ms_per_force_eval"], d["config"].get("fp64_rescan_fallbacks_in_timed_steps"),
          d["roofline"]["avg_launch_ms"])
PY
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/$out/trace224 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-exact-compare --direct-cus 224 > $GRAFT_REPO_ROOT/$out/trace224.log 2>&1); step $? trace224
python3 tools/step_timeline.py $out/trace224 | tail -30

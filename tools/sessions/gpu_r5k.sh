#!/bin/bash
# round 5, session k: k_pairs_cq as a persistent kernel (cells dealt by per-XCD counters), and the
# number of CUs it leaves to the reciprocal chain (CF_VARIANT_PAIR_FREE_CUS n: variants bits 12-18 =
# n + 1).  Expected: free 0 ~ the 1-cell-per-block kernel (181 us, balance slightly better);
# free 16-64: the DFT stages run beside the pair kernel (r5f/r5j timelines: they waited ~90-185
# us), step -20..-60 us.
out=gpurun_out/r5k
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
timeout -k 10 500 python -u -m pytest tests/test_gpu_cluster.py tests/test_gpu_half.py tests/test_gpu_overlap.py -x -q --timeout 200 --timeout-method thread > $out/gpu_tests.log 2>&1; step $? tests
tail -2 $out/gpu_tests.log
ARGS="--steps 40 --no-cpu-baseline --no-exact-compare"
for n in none 0 16 32 64; do
  if [ $n = none ]; then V=0; else V=$(( (n + 1) << 12 )); fi
  timeout -k 10 100 python -u bench.py $ARGS --variants $V > $out/bench_free$n.json 2> $out/bench_free$n.err; step $? free$n
done
python3 - <<'PY'
import json
for n in ("none", 0, 16, 32, 64):
    d = json.loads(open(f"gpurun_out/r5k/bench_free{n}.json").read().strip().splitlines()[-1])
    print(n, d["ms_per_step"], d.get("graph_replay_ms_per_step"), d["roofline"]["avg_launch_ms"], d["roofline"]["isolated"]["avg_launch_ms"],
          d["config"].get("fp64_rescan_fallbacks_in_timed_steps"))
PY
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/$out/trace32 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-exact-compare --variants $(( 33 << 12 )) > $GRAFT_REPO_ROOT/$out/trace32.log 2>&1); step $? trace32
python3 tools/step_timeline.py $out/trace32 | tail -26

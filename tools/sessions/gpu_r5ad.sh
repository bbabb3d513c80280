#!/bin/bash
# round 5, session ad: k_g_spread_mfma capped at 96 VGPRs (amdgpu_waves_per_eu(5): five blocks per CU
# instead of four; 24 B/lane of spills outside the MFMA group loop).  Expected: the per-tile source
# prologues of more blocks overlap the MFMAs: spread 77 -> ~70 us; bitwise the same.
out=gpurun_out/r5ad
mkdir -p $out
R=$GRAFT_REPO_ROOT
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_grid.py -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1; step $? tests
tail -1 $out/tests.log
ARGS="--steps 40 --no-cpu-baseline --no-exact-compare"
for i in 1 2 3; do
  timeout -k 10 100 python -u bench.py $ARGS > $out/bench$i.json 2> $out/bench$i.err; step $? bench$i
  python3 -c "
import json; d = json.loads(open('$out/bench$i.json').read().strip().splitlines()[-1])
print('c3', d['ms_per_step'], d.get('graph_replay_ms_per_step'), round(d['roofline']['avg_launch_ms'], 4))"
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$out/trace -o run --output-format csv -- python3 $R/bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-exact-compare > $R/$out/trace.log 2>&1); step $? trace
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r5ad/trace/**/*kernel_trace.csv", recursive=True)[0]
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(f)))
d = [(e[1] - e[0]) / 1e3 for e in ev if "spread_mfma" in e[2]]
print("k_g_spread_mfma, breakdown pass (alone): mean %.1f us" % (sum(d[5:45]) / 40), [round(x, 1) for x in d[5:15]])
PY

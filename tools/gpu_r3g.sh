#!/bin/bash
# GPU session (round 3): spread with zero-padded staging + fixed-offset reads, interpolation
# staging addresses; bitwise A/B of the spread forms, grid/overlap/config tests, isolated kernel
# times (default, CF_SPREAD_PASS=64), C3 bench.  Each GPU step time-limited; stops at the first
# step that faults, aborts or times out.
out=gpurun_out/r3g
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
CF_SPREAD_DPP=0 timeout -k 10 300 python -u tools/ab_bits.py run openmm-chargeflux_amd/libchargeflux_hip.so $out/ab0.npz > $out/ab0.log 2>&1; step $? ab0
timeout -k 10 300 python -u tools/ab_bits.py run openmm-chargeflux_amd/libchargeflux_hip.so $out/ab1.npz > $out/ab1.log 2>&1; step $? ab1
python tools/ab_bits.py cmp $out/ab0.npz $out/ab1.npz > $out/ab.txt 2>&1; echo "ab cmp rc=$?"; tail -2 $out/ab.txt
rm -f $out/ab0.npz $out/ab1.npz
timeout -k 10 900 python -u -m pytest tests/test_gpu_grid.py tests/test_gpu_overlap.py tests/test_gpu_configs.py tests/test_gpu_mixed.py -q \
    --timeout 300 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; echo "tests rc=$rc"; [ $rc -le 1 ] || exit $rc
R=$GRAFT_REPO_ROOT
ARGS="--steps 10 --warmup 3 --no-cpu-baseline --no-exact-compare"
cd /tmp && export TMPDIR=/tmp
CF_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$out/tr_new -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/$out/tr_new.log 2>&1; step $? tr_new
CF_OVERLAP=0 CF_SPREAD_PASS=64 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$out/tr_p64 -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/$out/tr_p64.log 2>&1; step $? tr_p64
cd $R
echo "== default (isolated)"; python3 tools/prof_stats.py $out/tr_new/run_kernel_stats.csv 8
echo "== pass 64 (isolated)"; python3 tools/prof_stats.py $out/tr_p64/run_kernel_stats.csv 8
timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-exact-compare > $out/bench.json 2> $out/bench.err; step $? bench
python - <<'P'
import json
d = json.loads(open("gpurun_out/r3g/bench.json").read().strip().splitlines()[-1])
print(d["ms_per_step"], d["ms_per_force_eval"], d["graph_replay_ms_per_step"], d["roofline"]["avg_launch_ms"], d["roofline"].get("isolated"))
print(d["kernels_ms_per_step"])
P
exit 0

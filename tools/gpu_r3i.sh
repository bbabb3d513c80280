#!/bin/bash
# GPU session (round 3): list builder A/B (per-candidate emission vs CF_NLIST_MASKS=1: same list,
# same bits), full GPU suite, isolated kernel times of both builder forms, C3 bench, W = 8 probe.
# Each GPU step time-limited; stops at the first step that faults, aborts or times out.
out=gpurun_out/r3i
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
CF_NLIST_MASKS=1 timeout -k 10 300 python -u tools/ab_bits.py run openmm-chargeflux_amd/libchargeflux_hip.so $out/ab0.npz > $out/ab0.log 2>&1; step $? ab0
timeout -k 10 300 python -u tools/ab_bits.py run openmm-chargeflux_amd/libchargeflux_hip.so $out/ab1.npz > $out/ab1.log 2>&1; step $? ab1
python tools/ab_bits.py cmp $out/ab0.npz $out/ab1.npz > $out/ab.txt 2>&1; echo "ab cmp rc=$?"; tail -2 $out/ab.txt
rm -f $out/ab0.npz $out/ab1.npz
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; echo "tests rc=$rc"; [ $rc -le 1 ] || exit $rc
R=$GRAFT_REPO_ROOT
ARGS="--steps 10 --warmup 3 --no-cpu-baseline --no-exact-compare"
cd /tmp && export TMPDIR=/tmp
CF_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$out/tr_iso -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/$out/tr_iso.log 2>&1; step $? tr_iso
CF_OVERLAP=0 CF_NLIST_MASKS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$out/tr_masks -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/$out/tr_masks.log 2>&1; step $? tr_masks
cd $R
echo "== isolated"; python3 tools/prof_stats.py $out/tr_iso/run_kernel_stats.csv 10
echo "== isolated, hit-mask builder"; python3 tools/prof_stats.py $out/tr_masks/run_kernel_stats.csv 6
timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-exact-compare > $out/bench.json 2> $out/bench.err; step $? bench
python - <<'P'
import json
d = json.loads(open("gpurun_out/r3i/bench.json").read().strip().splitlines()[-1])
print(d["ms_per_step"], d["ms_per_force_eval"], d["graph_replay_ms_per_step"], d["roofline"]["avg_launch_ms"], d["roofline"].get("isolated"))
print(d["kernels_ms_per_step"])
P
timeout -k 10 300 python -u tools/scaling_probe.py --worlds 8 --no-timing > $out/probe.json 2> $out/probe.err; step $? probe
cut -c1-120 $out/probe.json
exit 0

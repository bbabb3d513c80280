#!/bin/bash
# GPU session (round 3): LJ-first rows + wave-uniform LJ skip in the pair kernels; full GPU test
# suite, isolated kernel times (CF_OVERLAP=0) of the current tree, C3 bench.  Each GPU step
# time-limited; stops at the first step that faults, aborts or times out.
out=gpurun_out/r3h
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
# list builder: per-candidate emission (default) vs the hit-mask form (CF_NLIST_MASKS=1): same list, same bits
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
CF_OVERLAP=0 timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d $R/$out/pmc_a -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/$out/pmc_a.log 2>&1; step $? pmc_a
cd $R
python3 tools/pmc_summary.py $out/summary.json $out/tr_iso/run_kernel_trace.csv $out/pmc_a/run_counter_collection.csv > $out/summary.txt
head -6 $out/summary.txt | cut -c1-300
echo "== isolated"; python3 tools/prof_stats.py $out/tr_iso/run_kernel_stats.csv 24
echo "== isolated, hit-mask builder"; python3 tools/prof_stats.py $out/tr_masks/run_kernel_stats.csv 6
timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-exact-compare > $out/bench.json 2> $out/bench.err; step $? bench
python - <<'P'
import json
d = json.loads(open("gpurun_out/r3h/bench.json").read().strip().splitlines()[-1])
print(d["ms_per_step"], d["ms_per_force_eval"], d["graph_replay_ms_per_step"], d["roofline"]["avg_launch_ms"], d["roofline"].get("isolated"))
print(d["kernels_ms_per_step"])
P
timeout -k 10 300 python -u tools/scaling_probe.py --worlds 1 8 --no-timing > $out/probe.json 2> $out/probe.err; step $? probe
cut -c1-120 $out/probe.json
# accuracy / speed of the kernel width: W = 13 and 14 with the exact k-sum comparison
for w in 13 14; do
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --grid-width $w > $out/bench_w$w.json 2> $out/bench_w$w.err; step $? bench_w$w
done
python - <<'P'
import json
for w in (13, 14):
    d = json.loads(open(f"gpurun_out/r3h/bench_w{w}.json").read().strip().splitlines()[-1])
    print(w, d["ms_per_step"], d["exact_kspace"], {k: d["kernels_ms_per_step"][k] for k in ("grid_sort", "grid_spread", "grid_interp")})
P
# C5 (768k atoms, mixed precision): the BASELINE config-5 workload on one GPU
timeout -k 10 600 python -u bench.py --config C5 --precision mixed --steps 10 --warmup 3 --no-cpu-baseline --no-exact-compare > $out/bench_c5.json 2> $out/bench_c5.err; step $? bench_c5
python - <<'P'
import json
d = json.loads(open("gpurun_out/r3h/bench_c5.json").read().strip().splitlines()[-1])
print("C5", d["ms_per_step"], d["value"], d["kernels_ms_per_step"])
P
exit 0

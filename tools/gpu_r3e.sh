#!/bin/bash
# GPU session (round 3, spread DPP change, interpolation reduction): bitwise A/B of the spread's
# DPP form against the scalar-load form (CF_SPREAD_DPP=0) on tools/ab_bits.py's cases, the GPU tests, C3 bench lines
# for both forms, kernel stats, FETCH/WRITE calibration passes.  Each GPU step has its own time
# limit; the script stops at the first step that faults, aborts or times out.
out=gpurun_out/r3e
mkdir -p $out
set -o pipefail
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
CF_SPREAD_DPP=0 timeout -k 10 300 python -u tools/ab_bits.py run openmm-chargeflux_amd/libchargeflux_hip.so $out/ab0.npz > $out/ab0.log 2>&1; step $? ab0
timeout -k 10 300 python -u tools/ab_bits.py run openmm-chargeflux_amd/libchargeflux_hip.so $out/ab1.npz > $out/ab1.log 2>&1; step $? ab1
python tools/ab_bits.py cmp $out/ab0.npz $out/ab1.npz > $out/ab.txt 2>&1; echo "ab cmp rc=$?"; cat $out/ab.txt
rm -f $out/ab0.npz $out/ab1.npz
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $out/tests_gpu.log 2>&1
rc=$?; tail -3 $out/tests_gpu.log; echo "tests_gpu rc=$rc"; [ $rc -le 1 ] || exit $rc   # a plain test failure continues
timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-exact-compare > $out/bench_dpp.json 2> $out/bench_dpp.err; step $? bench_dpp
CF_SPREAD_DPP=0 timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-exact-compare > $out/bench_scalar.json 2> $out/bench_scalar.err; step $? bench_scalar
python - <<'E'
import json
for f in ("bench_dpp", "bench_scalar"):
    d = json.loads(open(f"gpurun_out/r3e/{f}.json").read().strip().splitlines()[-1])
    print(f, d["ms_per_step"], d["ms_per_force_eval"], {k: d["kernels_ms_per_step"][k] for k in ("grid_spread", "grid_interp", "direct_pairs", "grid_sort")})
E
timeout -k 10 300 python -u tools/scaling_probe.py --worlds 1 2 4 8 --no-timing > $out/probe_ovl.json 2> $out/probe_ovl.err; step $? probe_ovl
CF_OVERLAP=0 timeout -k 10 300 python -u tools/scaling_probe.py --worlds 8 --no-timing > $out/probe_1s.json 2> $out/probe_1s.err; step $? probe_1s
cat $out/probe_ovl.json $out/probe_1s.json | cut -c1-200
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$out/trace -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-exact-compare > $R/$out/trace.log 2>&1; step $? trace
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d $R/$out/cal_f -o run --output-format csv -- $R/tools/fetch_calib > $R/$out/cal_f.log 2>&1; step $? cal_f
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -d $R/$out/cal_w -o run --output-format csv -- $R/tools/fetch_calib > $R/$out/cal_w.log 2>&1; step $? cal_w
cd $R
python3 tools/prof_stats.py $out/trace/run_kernel_stats.csv 2>/dev/null | head -30 || true
exit 0

#!/bin/bash
# round 4 final at HEAD: full GPU suite, smoke, the default bench (with the CPU baseline), the
# bench command under rocprofv3 --kernel-trace --stats, C5 mixed bench.
out=gpurun_out/r4z
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
R=$GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $out/gpu_tests.log 2>&1; rc=$?; tail -2 $out/gpu_tests.log; step $rc gpu_tests
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1; step $? smoke
timeout -k 10 600 python -u bench.py > $out/bench_c3.json 2> $out/bench_c3.err; step $? bench_c3
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$out/tr -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-exact-compare > $R/$out/tr.log 2>&1); step $? tr
timeout -k 10 400 python -u bench.py --config C5 --precision mixed --steps 10 --warmup 3 --no-cpu-baseline > $out/bench_c5.json 2> $out/bench_c5.err; step $? bench_c5

#!/bin/bash
# round 4 closing check at HEAD: full GPU suite and smoke.
out=gpurun_out/r4ae
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $out/gpu_tests.log 2>&1; rc=$?; tail -2 $out/gpu_tests.log; step $rc gpu_tests
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1; step $? smoke
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-exact-compare > $out/bench.json 2> $out/bench.err; step $? bench
tail -1 $out/bench.json | cut -c1-250

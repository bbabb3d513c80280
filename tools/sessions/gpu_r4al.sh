#!/bin/bash
# round 4 closing check at HEAD after the W <= 9 tap-row change: full GPU suite, smoke, C3 bench.
out=gpurun_out/r4al
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1; rc=$?; tail -2 $out/tests.log; step $rc tests
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1; rc=$?; tail -1 $out/smoke.log; step $rc smoke
timeout -k 10 400 python -u bench.py > $out/bench.json 2> $out/bench.err; step $? bench
python3 -c "import json; d = json.loads(open('$out/bench.json').read().strip().splitlines()[-1]); print('bench', d['ms_per_step'], d['value'], d['roofline']['frac'])"

#!/bin/bash
# round 4: the full GPU suite on the current tree, then a C5 mixed bench with its breakdown.
out=gpurun_out/r4s
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $out/gpu_tests.log 2>&1; rc=$?; tail -3 $out/gpu_tests.log; step $rc gpu_tests
timeout -k 10 400 python -u bench.py --config C5 --precision mixed --steps 10 --warmup 3 --no-cpu-baseline --no-exact-compare > $out/c5.json 2> $out/c5.err; step $? c5
python3 -c "import json; d = json.loads(open('$out/c5.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d.get('graph_replay_ms_per_step'), d['kernels_ms_per_step'])"

#!/bin/bash
# GPU box: all -m gpu tests, the bench with and without per-kernel events, and a rocprofv3
# kernel trace of the bench (gpurun_out/prof_$1).  Every GPU step has its own time limit and
# the first failure ends the script.
set -e
TAG=${1:-r}
OUT=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $OUT/prof_$TAG
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/t_$TAG.log 2>&1
timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-exact-compare --steps 20 --warmup 5 --no-kernel-timing ${@:2} > $OUT/bench_nt_$TAG.json 2> $OUT/bench_nt_$TAG.err
timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 ${@:2} > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err
cd /tmp
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof_$TAG -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-exact-compare --steps 10 --warmup 2 ${@:2} > $OUT/prof_$TAG/log.txt 2>&1

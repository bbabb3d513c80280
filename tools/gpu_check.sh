#!/bin/bash
# GPU box: all -m gpu tests, smoke, the default bench line and a rocprofv3 kernel trace of it
# (gpurun_out/<tag>/).  Every GPU step has its own time limit; the first failure ends the script.
set -e
TAG=${1:-r02}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -k 10 300 python -u bench.py ${@:2} > $OUT/bench.json 2> $OUT/bench.err
cd /tmp
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-exact-compare --steps 10 --warmup 2 ${@:2} > $OUT/prof.log 2>&1

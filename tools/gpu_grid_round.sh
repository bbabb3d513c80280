#!/bin/bash
# GPU box: grid-path tests + a rocprofv3 kernel-trace of the grid-path bench (gpurun_out/prof_$1)
set -e
TAG=${1:-g}
OUT=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $OUT/prof_$TAG
timeout -k 10 400 python -u -m pytest tests/test_gpu_grid.py -x -q --timeout 200 --timeout-method thread > $OUT/tg_$TAG.log 2>&1
cd /tmp
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof_$TAG -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --kspace-algo 2 --no-cpu-baseline --no-exact-compare --steps 10 --warmup 2 ${@:2} > $OUT/prof_$TAG/log.txt 2>&1

#!/bin/bash
# One rocprofv3 --pmc pass over a short grid-path bench, restricted to kernels matching $2.
# usage: tools/pmc_one.sh TAG REGEX COUNTERS...   (GPU box, repo root)
set -e
TAG=$1; RX=$2; shift 2
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex "$RX" -d $OUT -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --kspace-algo 2 --no-cpu-baseline --steps 3 --warmup 1 > $OUT/log.txt 2>&1

#!/bin/bash
# GPU box: rocprofv3 kernel traces of the C3 and C5 (mixed) bench, per-kernel stats
set -e
cd /tmp
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-pd}
mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/c3 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-exact-compare --no-kernel-timing --steps 10 --warmup 2 > $OUT/c3.json 2> $OUT/c3.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/c5 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config C5 --precision mixed --no-cpu-baseline --no-exact-compare --no-kernel-timing --steps 5 --warmup 2 > $OUT/c5.json 2> $OUT/c5.err

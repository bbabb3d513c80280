#!/bin/bash
# GPU box: the grid tests (factorized DFT vs GEMM stages, oracle parity) and the C3 / C5 bench
# lines with per-phase times.  Each GPU step has its own limit; the first failure ends it.
set -e
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-d8}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_grid.py -x -v --timeout 200 --timeout-method thread > $OUT/t_grid.log 2>&1
timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > $OUT/c3.json 2> $OUT/c3.err
timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-exact-compare --no-kernel-timing --steps 100 --warmup 5 > $OUT/c3_nt.json 2> $OUT/c3_nt.err
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-exact-compare --config C5 --precision mixed --steps 10 --warmup 3 > $OUT/c5.json 2> $OUT/c5.err

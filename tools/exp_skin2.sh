#!/bin/bash
# GPU box: C3 bench (no per-kernel events, 100 steps) at several neighbour skins
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/skin2
for s in ${SKINS:-0.08 0.1 0.12 0.15 0.1}; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-exact-compare --no-kernel-timing --steps 100 --warmup 5 --neighbor-skin $s > gpurun_out/skin2/s$s.json 2> gpurun_out/skin2/s$s.err
done

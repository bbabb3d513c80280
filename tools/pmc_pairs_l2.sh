#!/bin/bash
# GPU box: L1/L2 request counters of the half-list pair kernel (C3 bench), separate passes
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_${1:-pl2}
mkdir -p $OUT
cd /tmp
export TMPDIR=/tmp
B="$GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-exact-compare --no-kernel-timing --steps 3 --warmup 1"
timeout -s KILL 120 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum --kernel-include-regex "pairs_half|nlist_wave|g_interp|g_spread" -d $OUT/a -o run --output-format csv -- python3 $B > $OUT/a.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum TA_BUSY_avr TA_BUSY_max --kernel-include-regex "pairs_half|nlist_wave|g_interp|g_spread" -d $OUT/b -o run --output-format csv -- python3 $B > $OUT/b.log 2>&1
cd $GRAFT_REPO_ROOT
for p in a b; do python3 tools/pmc_show.py $OUT/$p; done > $OUT/summary.txt

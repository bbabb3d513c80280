# GPU box: kernel trace of the C5 mixed-precision bench
set -e
cd /tmp
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/c5prof
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config C5 --precision mixed --no-cpu-baseline --no-exact-compare --steps 5 --warmup 2 > $OUT/bench.json 2> $OUT/bench.err

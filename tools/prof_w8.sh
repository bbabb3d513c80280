# GPU box: kernel trace of rank 0 of an 8-way decomposition of C3 (tools/scaling_probe.py)
set -e
cd /tmp
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/w8
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/scaling_probe.py --worlds 8 --steps 20 > $OUT/probe.txt 2> $OUT/probe.err

#!/bin/bash
# round 4: rehearsal of the multi-rank bench path (2 and 4 processes on the one GPU, gloo for the
# collectives; CF_BENCH_ONE_GPU=1) with the round-4 hand-overs -- not a benchmark configuration.
out=gpurun_out/r4w
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
for n in 2 4; do
    CF_BENCH_ONE_GPU=1 CF_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2951$n bench.py --gpus $n --steps 5 --warmup 2 > $out/mr_$n.json 2> $out/mr_$n.err; step $? mr_$n
    tail -1 $out/mr_$n.json | cut -c1-300
done

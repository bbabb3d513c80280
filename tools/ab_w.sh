set -e
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/abw
mkdir -p $OUT
for W in 14 12 13; do
timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 40 --warmup 5 --grid-width $W > $OUT/w$W.json 2> $OUT/w$W.err
done
timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-exact-compare --no-kernel-timing --steps 100 --warmup 5 --grid-width 12 > $OUT/w12_nt.json 2>> $OUT/w12.err
timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-exact-compare --no-kernel-timing --steps 100 --warmup 5 --grid-width 14 > $OUT/w14_nt.json 2>> $OUT/w14.err

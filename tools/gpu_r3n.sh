#!/bin/bash
# GPU session (round 3): same-box A/B of the half-list pair kernel, walk_row (4-8 lanes per row,
# this tree) against the previous one-sub-list-per-lane walk (tmp_ab/libchargeflux_hip_old.so,
# built from the previous commit's cf_kernels_core.hip): isolated kernel times and C3 bench,
# alternated.  Each GPU step time-limited.
out=gpurun_out/r3n
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
L=openmm-chargeflux_amd/libchargeflux_hip.so
cp $L tmp_ab/libchargeflux_hip_new.so
use() { cp tmp_ab/libchargeflux_hip_$1.so $L; }
R=$GRAFT_REPO_ROOT
ARGS="--steps 10 --warmup 3 --no-cpu-baseline --no-exact-compare"
for v in new old; do
    use $v
    (cd /tmp && export TMPDIR=/tmp && CF_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$out/tr_$v -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/$out/tr_$v.log 2>&1); step $? tr_$v
done
for v in new old; do echo "== $v"; python3 tools/prof_stats.py $out/tr_$v/run_kernel_stats.csv 3; done
for n in new1 old1 new2 old2; do
    use ${n%?}
    timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-exact-compare > $out/bench_$n.json 2> $out/bench_$n.err; step $? bench_$n
done
use new
python - <<'P'
import json
for n in ("new1", "old1", "new2", "old2"):
    d = json.loads(open(f"gpurun_out/r3n/bench_{n}.json").read().strip().splitlines()[-1])
    print(n, d["ms_per_step"], d["ms_per_force_eval"], d["roofline"]["isolated"]["avg_launch_ms"])
P
exit 0

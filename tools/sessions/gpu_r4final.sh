#!/bin/bash
# round 4 evidence: smoke, the default bench (C3, CPU baseline included), the rocprofv3 trace +
# PMC passes of the same bench command (tools/profile_round.sh), the C5 mixed bench.
out=gpurun_out/r4final
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1; step $? smoke
timeout -k 10 600 python -u bench.py > $out/bench_c3.json 2> $out/bench_c3.err; step $? bench_c3
tail -1 $out/bench_c3.json | cut -c1-400
timeout -k 10 900 bash tools/profile_round.sh r04 > $out/profile.log 2>&1; step $? profile
timeout -k 10 400 python -u bench.py --config C5 --precision mixed --steps 10 --warmup 3 --no-cpu-baseline > $out/bench_c5.json 2> $out/bench_c5.err; step $? bench_c5
tail -1 $out/bench_c5.json | cut -c1-300

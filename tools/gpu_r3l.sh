#!/bin/bash
# GPU session (round 3): k_g_interp4 (W <= 8) parity, then the C5 mixed-precision bench with
# CF_INTERP4 on and off.  Each GPU step time-limited.
out=gpurun_out/r3l
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_grid.py -m gpu -q -k "interp" --timeout 120 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1; r=$?
tail -3 $out/tests.log; step $r tests
for v in 1 0; do
    CF_INTERP4=$v timeout -k 10 600 python -u bench.py --config C5 --precision mixed --steps 10 --warmup 3 --no-cpu-baseline --no-exact-compare > $out/c5_i4_$v.json 2> $out/c5_i4_$v.err; step $? c5_i4_$v
done
python - <<'P'
import json
for v in ("1", "0"):
    d = json.loads(open(f"gpurun_out/r3l/c5_i4_{v}.json").read().strip().splitlines()[-1])
    k = d["kernels_ms_per_step"]
    print("interp4", v, d["ms_per_step"], d["value"], k["grid_interp"], k["grid_spread"])
P
exit 0

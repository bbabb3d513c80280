#!/bin/bash
# One GPU session: GPU test suite, bitwise A/B against a stored build, smoke, a short bench.
# Usage: tools/gpu_r3.sh OUTDIR [OLD_LIB]   (run from the repo root; each step time-limited;
# stops at the first step that faults, aborts or times out -- a plain test failure continues)
out=${1:-gpurun_out/r3}
old=${2:-}
mkdir -p "$out"
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > "$out/tests.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 "$out/tests.log"; ok $rc || exit $rc
if [ -n "$old" ]; then
    timeout -k 10 300 python -u tools/ab_bits.py run "$old" "$out/ab_old.npz" > "$out/ab.log" 2>&1 || exit $?
    timeout -k 10 300 python -u tools/ab_bits.py run openmm-chargeflux_amd/libchargeflux_hip.so "$out/ab_new.npz" >> "$out/ab.log" 2>&1 || exit $?
    python tools/ab_bits.py cmp "$out/ab_old.npz" "$out/ab_new.npz" >> "$out/ab.log" 2>&1; echo "ab rc=$?"; tail -3 "$out/ab.log"
    rm -f "$out/ab_old.npz" "$out/ab_new.npz"
fi
if [ -n "$PROBES" ]; then
    for pr in $PROBES; do
        timeout -k 10 600 python -u "$pr" > "$out/$(basename "$pr" .py).json" 2> "$out/$(basename "$pr" .py).err"
        rc=$?; echo "$pr rc=$rc"; tail -c 800 "$out/$(basename "$pr" .py).json"; [ $rc -eq 0 ] || exit $rc
    done
fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 "$out/smoke.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$out/bench.json" 2> "$out/bench.err"
rc=$?; echo "bench rc=$rc"; tail -c 600 "$out/bench.json"; exit $rc

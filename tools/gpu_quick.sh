#!/bin/bash
# Quick GPU session: selected test files, optional probes, a bench line.  Each GPU step has its
# own time limit; stops after a fault / abort / timeout (a plain test failure continues).
# Usage: TESTS="tests/a.py tests/b.py" PROBES="tools/x.py" BENCH="--steps 20 ..." tools/gpu_quick.sh OUTDIR
out=${1:-gpurun_out/q}
mkdir -p "$out"
if [ -n "$TESTS" ]; then
    timeout -k 10 900 python -u -m pytest $TESTS -q --timeout 300 --timeout-method thread -p no:cacheprovider \
        > "$out/tests.log" 2>&1
    rc=$?; echo "tests rc=$rc"; tail -8 "$out/tests.log"; { [ $rc -eq 0 ] || [ $rc -eq 1 ]; } || exit $rc
fi
for pr in $PROBES; do
    b=$(basename "$pr" .py)
    timeout -k 10 600 python -u $pr > "$out/$b.json" 2> "$out/$b.err"
    rc=$?; echo "$pr rc=$rc"; tail -c 1500 "$out/$b.json"; [ $rc -eq 0 ] || exit $rc
done
if [ -n "$BENCH" ]; then
    timeout -k 10 600 python -u bench.py $BENCH > "$out/bench.json" 2> "$out/bench.err"
    rc=$?; echo "bench rc=$rc"; tail -c 2500 "$out/bench.json"; [ $rc -eq 0 ] || exit $rc
fi
exit 0

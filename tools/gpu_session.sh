#!/bin/bash
# One GPU session on the gpurun box (replaces the per-session scripts of rounds 4-5).
#
#   tools/gpu_session.sh TAG STEP [STEP ...]
#
# Every step runs under its own time limit; the first failing step ends the session (no GPU
# step runs after a fault, an abort or a time limit).  Output goes to gpurun_out/TAG/.  A
# failing step's whole log is also copied to profiles/TAG_FAILED_<step>.log, so a retry never
# overwrites the evidence of a failure.
#
# Steps:
#   tests[=EXPR]      pytest -m gpu (optionally -k EXPR), one process, per-test timeout
#   smoke             __graft_entry__.smoke()
#   bench_c3 / bench_c5 / bench_c3_mixed   the bench line (JSON) of that configuration
#   trace_c3 / trace_c5                    rocprofv3 --kernel-trace --stats of the bench command
#   pmc_c3 / pmc_c5                        three separate --pmc passes of the bench command +
#                                          tools/pmc_summary.py (needs trace_<cfg> first)
#   py=SCRIPT[:ARGS]  python -u SCRIPT ARGS (a probe under tools/), output in TAG/SCRIPT.log
#   trace_py=SCRIPT[:ARGS]                 rocprofv3 --kernel-trace --stats of such a probe
#   (ARGS: comma-separated, e.g. py=tools/scaling_probe.py:--worlds,1,8,--no-timing)
set -o pipefail
TAG=$1; shift
out=gpurun_out/$TAG
mkdir -p $out profiles
R=${GRAFT_REPO_ROOT:-$(pwd)}
fail() {   # step name, log file, rc
    echo "STEP $1 FAILED rc=$3 (log kept as profiles/${TAG}_FAILED_$1.log and $out/FAILED_$1.log)"
    [ -f "$2" ] && cp "$2" "profiles/${TAG}_FAILED_$1.log"
    # (gpurun merges only gpurun_out/ back from the box: this copy is the one that returns)
    [ -f "$2" ] && cp "$2" "$out/FAILED_$1.log"
    exit $3
}
run() {   # name, log, seconds, command...
    local name=$1 log=$2 secs=$3; shift 3
    local t0=$(date +%s)
    timeout -k 10 $secs "$@" > $log 2>&1
    local rc=$?
    echo "STEP $name rc=$rc $(( $(date +%s) - t0 ))s"
    [ $rc -eq 0 ] || fail $name $log $rc
}
cfgargs() { case $1 in c5) echo "--config C5 --precision mixed";; c3_mixed) echo "--precision mixed";; *) echo "";; esac; }
# (the C5 CPU-baseline sample runs minutes without output: the box's silence guard would kill it)
benchargs() { case $1 in c5) echo "--no-cpu-baseline";; *) echo "";; esac; }
PROF_ARGS="--steps 5 --warmup 2 --no-cpu-baseline --no-exact-compare"
for st in "$@"; do
    case $st in
    tests|tests=*)
        k=(); [ "$st" != tests ] && k=(-k "${st#tests=}")   # (an array: the expression may hold spaces)
        run tests $out/gpu_tests.log 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${k[@]}"
        tail -2 $out/gpu_tests.log;;
    smoke)
        run smoke $out/smoke.log 200 python -u -c "import __graft_entry__ as g; g.smoke()"
        tail -3 $out/smoke.log;;
    bench=*)   # bench=ARGS (comma-separated): one bench line with these arguments
        a=${st#bench=}; tagf=$(echo "$a" | tr -c 'A-Za-z0-9.' '_')
        timeout -k 10 400 python -u bench.py ${a//,/ } > $out/bench_$tagf.json 2> $out/bench_$tagf.err
        rc=$?; echo "STEP bench $a rc=$rc"; [ $rc -eq 0 ] || fail bench_$tagf $out/bench_$tagf.err $rc
        python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d.get('graph_replay_ms_per_step'))" $out/bench_$tagf.json "$a";;
    bench_*)
        cfg=${st#bench_}
        timeout -k 10 400 python -u bench.py $(cfgargs $cfg) $(benchargs $cfg) > $out/$st.json 2> $out/$st.err
        rc=$?; echo "STEP $st rc=$rc"; [ $rc -eq 0 ] || fail $st $out/$st.err $rc
        tail -c 2500 $out/$st.json; echo;;
    trace_py=*)   # rocprofv3 --kernel-trace --stats of a probe: trace_py=SCRIPT[:ARGS]
        spec=${st#trace_py=}; script=${spec%%:*}; args=""; [ "$spec" != "$script" ] && args=${spec#*:}
        name=trace_$(basename $script .py)
        (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$out/$name -o run \
            --output-format csv -- python3 $R/$script ${args//,/ } > $R/$out/$name.log 2>&1)
        rc=$?; echo "STEP $st rc=$rc"; [ $rc -eq 0 ] || fail $name $out/$name.log $rc
        python3 tools/prof_stats.py $out/$name/run_kernel_stats.csv 2>/dev/null | head -30;;
    trace_*)
        cfg=${st#trace_}
        (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$out/trace_$cfg -o run \
            --output-format csv -- python3 $R/bench.py $PROF_ARGS $(cfgargs $cfg) > $R/$out/trace_$cfg.log 2>&1)
        rc=$?; echo "STEP $st rc=$rc"; [ $rc -eq 0 ] || fail $st $out/trace_$cfg.log $rc
        python3 tools/prof_stats.py $out/trace_$cfg/run_kernel_stats.csv 2>/dev/null | head -25;;
    pmc_*)
        cfg=${st#pmc_}
        i=0
        for ctr in "SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" FETCH_SIZE WRITE_SIZE; do
            i=$((i + 1))
            (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --pmc $ctr -d $R/$out/pmc${i}_$cfg -o run \
                --output-format csv -- python3 $R/bench.py $PROF_ARGS $(cfgargs $cfg) > $R/$out/pmc${i}_$cfg.log 2>&1)
            rc=$?; echo "STEP ${st}_$i rc=$rc"; [ $rc -eq 0 ] || fail ${st}_$i $out/pmc${i}_$cfg.log $rc
        done
        python3 tools/pmc_summary.py $out/summary_$cfg.json $out/trace_$cfg/run_kernel_trace.csv \
            $out/pmc1_$cfg/run_counter_collection.csv $out/pmc2_$cfg/run_counter_collection.csv \
            $out/pmc3_$cfg/run_counter_collection.csv > $out/summary_$cfg.txt 2>&1
        head -14 $out/summary_$cfg.txt;;
    py=*)
        spec=${st#py=}; script=${spec%%:*}; args=""; [ "$spec" != "$script" ] && args=${spec#*:}
        name=$(basename $script .py)
        run $name $out/$name.log 600 python -u $script ${args//,/ }
        tail -40 $out/$name.log;;
    *) echo "unknown step $st"; exit 2;;
    esac
done
echo "SESSION $TAG done"

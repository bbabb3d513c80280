#!/bin/bash
# round 4: cluster-pair kernel counters.  Parity first (test_gpu_cluster), then an isolated
# kernel trace and one SQ counter pass for k_pairs_cq / k_cl_build and, with CF_CLUSTER=0, the
# per-atom half list's k_pairs_half / k_nlist_wave on the same bench.
out=gpurun_out/r4c
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_cluster.py tests/test_gpu_half.py tests/test_gpu_mixed.py -x -q --timeout 150 --timeout-method thread > $out/tests.log 2>&1; rc=$?; tail -3 $out/tests.log; step $rc tests
R=$GRAFT_REPO_ROOT
(cd /tmp && export TMPDIR=/tmp && CF_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$out/tr -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-exact-compare > $R/$out/tr.log 2>&1); step $? trace
SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT"
for v in cq half; do
    if [ $v = half ]; then export CF_CLUSTER=0; fi
    (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $SQ --kernel-include-regex "k_pairs|k_cl_build|k_nlist_wave" -d $R/$out/pmc_$v -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-exact-compare --no-kernel-timing > $R/$out/pmc_$v.log 2>&1); step $? pmc_$v
    (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_avr TA_BUSY_max SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE --kernel-include-regex "k_pairs|k_cl_build|k_nlist_wave" -d $R/$out/pmc2_$v -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-exact-compare --no-kernel-timing > $R/$out/pmc2_$v.log 2>&1); step $? pmc2_$v
done
unset CF_CLUSTER
for v in cq half; do echo "== $v"; python3 tools/pmc_show.py $out/pmc_$v; python3 tools/pmc_show.py $out/pmc2_$v; done > $out/pmc.txt 2>&1
cat $out/pmc.txt
python3 - <<'P'
import csv
rows = list(csv.DictReader(open("gpurun_out/r4c/tr/run_kernel_stats.csv")))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:12]:
    print(r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1000, 1), "max", round(float(r["MaxNs"]) / 1000, 1))
P

#!/bin/bash
# round 5, session g: counters of k_pairs_es (octant) against k_pairs_cq (18-cell) at C3 -- the
# octant kernel ran 236 us against 181 (r5f).  Expected: either more VALU per pair (short rows'
# partial phase-B steps) or more wait cycles (the per-row load chain, 23 rows per wave vs 3).
out=gpurun_out/r5g
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
R=$GRAFT_REPO_ROOT
for pl in octant cluster; do
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --kernel-include-regex "k_pairs" -d $R/$out/pmc_$pl -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-exact-compare --pair-list $pl > $R/$out/pmc_$pl.log 2>&1); step $? pmc_$pl
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS --kernel-include-regex "k_pairs" -d $R/$out/pmc2_$pl -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-exact-compare --pair-list $pl > $R/$out/pmc2_$pl.log 2>&1); step $? pmc2_$pl
done
python3 - <<'PY'
import csv, collections
for pl in ("octant", "cluster"):
    for d in ("pmc", "pmc2"):
        per = collections.defaultdict(float); n = collections.Counter()
        disp = set()
        for r in csv.DictReader(open(f"gpurun_out/r5g/{d}_{pl}/run_counter_collection.csv")):
            per[r["Counter_Name"]] += float(r["Counter_Value"]); disp.add(r["Dispatch_Id"])
        nd = len(disp)
        print(pl, d, nd, {k: f"{v / nd:.3e}" for k, v in sorted(per.items())})
PY

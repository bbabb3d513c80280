#!/bin/bash
# round 4: the cluster-pair list on several ranks (ownership-filtered half list): the multi-rank
# GPU tests, then rank-0 probes W = 1/2/4/8 against the full per-atom list (CF_CLUSTER_MR=0).
out=gpurun_out/r4ag
mkdir -p $out
step() { local rc=$1 name=$2; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_graph.py tests/test_gpu_grid.py tests/test_gpu_overlap.py tests/test_gpu_parity.py tests/test_gpu_skin.py tests/test_gpu_triclinic.py -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1; rc=$?; tail -3 $out/tests.log; step $rc tests
for v in cl full; do
    if [ $v = full ]; then export CF_CLUSTER_MR=0; else unset CF_CLUSTER_MR; fi
    timeout -k 10 400 python -u tools/scaling_probe.py --worlds 1 2 4 8 --steps 40 --neighbor-skin 0.15 --no-timing > $out/probe_$v.jsonl 2> $out/probe_$v.err; step $? probe_$v
    python3 -c "
import json
for l in open('$out/probe_$v.jsonl'):
    d = json.loads(l); print('$v W', d['world'], d['ms_per_step'])"
done

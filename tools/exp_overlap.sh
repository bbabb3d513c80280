# GPU box: reciprocal chain on a second stream (CF_OVERLAP) -- bitwise A/B against abl/head,
# bench timing both ways, the tests that touch the single-rank launch sequence
cd $GRAFT_REPO_ROOT
o=gpurun_out/ovl; mkdir -p $o
bash tools/ab_head.sh || exit 1
B="python -u bench.py --no-cpu-baseline --no-exact-compare --steps 40 --warmup 5"
for v in 1 0 1 0; do
  CF_OVERLAP=$v timeout -k 10 120 $B > $o/b_$v.json 2>$o/b_$v.err || { tail -5 $o/b_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$o/b_$v.json')); print('overlap=$v', d['ms_per_step'], d.get('ms_per_force_eval'), d.get('graph_replay_ms_per_step'))"
done
timeout -k 10 700 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_grid.py tests/test_gpu_half.py tests/test_gpu_parity.py tests/test_gpu_skin.py -x -q --timeout 200 --timeout-method thread > $o/tests.log 2>&1
rc=$?; tail -3 $o/tests.log; exit $rc

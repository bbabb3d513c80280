# GPU box: half-list tests, then half vs full list timing at C3
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_half.py -x -q --timeout 200 --timeout-method thread > gpurun_out/half_tests.log 2>&1 || { tail -30 gpurun_out/half_tests.log; exit 1; }
tail -2 gpurun_out/half_tests.log
B="python -u bench.py --no-cpu-baseline --no-exact-compare --steps 40 --warmup 5"
for h in 1 0 1; do
  CF_HALF=$h timeout -k 10 120 $B > gpurun_out/h_tmp.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/h_tmp.json')); k=d['kernels_ms_per_step']; print('half=$h', d['ms_per_step'], k['direct_pairs'], k['neighbor_list'], d['config']['nlist_builds_in_timed_steps'])"
done

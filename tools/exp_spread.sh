cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_grid.py tests/test_gpu_configs.py tests/test_gpu_mixed.py -x -q --timeout 200 --timeout-method thread > gpurun_out/exp_spread_tests.log 2>&1 || exit 1
B="python -u bench.py --no-cpu-baseline --no-exact-compare --steps 20 --warmup 5"
for cfg in "CF_EXP_OLD_SPREAD=1" "X=1"; do
  env $cfg timeout -k 10 120 $B > gpurun_out/sp_tmp.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/sp_tmp.json')); k=d['kernels_ms_per_step']; print('$cfg', d['ms_per_step'], k['grid_spread'])" >> gpurun_out/exp_spread.txt
done

# GPU box: grid-path tests, then the bench's per-phase timing at C3 (twice)
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_grid.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/grid_tests.log 2>&1 || { tail -30 gpurun_out/grid_tests.log; exit 1; }
tail -2 gpurun_out/grid_tests.log
B="python -u bench.py --no-cpu-baseline --no-exact-compare --steps 40 --warmup 5"
for r in 1 2; do
  timeout -k 10 120 $B > gpurun_out/g_tmp.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/g_tmp.json')); k=d['kernels_ms_per_step']; print(d['ms_per_step'], 'spread', k['grid_spread'], 'interp', k['grid_interp'], 'sort', k['grid_sort'], 'dft', k['grid_dft_fwd'], k['grid_dft_inv'])"
done

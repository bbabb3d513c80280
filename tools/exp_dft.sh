# GPU box: grid-path tests, C3 bench per-phase timing, C3 and C5 kernel traces (DFT stages)
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_grid.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/grid_tests.log 2>&1 || { tail -30 gpurun_out/grid_tests.log; exit 1; }
tail -2 gpurun_out/grid_tests.log
B="python -u bench.py --no-cpu-baseline --no-exact-compare --steps 40 --warmup 5"
for r in 1 2; do
  timeout -k 10 120 $B > gpurun_out/g_tmp.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/g_tmp.json')); k=d['kernels_ms_per_step']; print(d['ms_per_step'], 'spread', k['grid_spread'], 'interp', k['grid_interp'], 'sort', k['grid_sort'], 'dft', k['grid_dft_fwd'], k['grid_dft_inv'])"
done
cd /tmp && export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/dft
mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/c3 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-exact-compare --steps 20 --warmup 3 > $OUT/c3.json 2> $OUT/c3.err || exit 1
python3 $GRAFT_REPO_ROOT/tools/prof_stats.py $OUT/c3 40 | grep -i "cgemm\|coeffs"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/c5 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config C5 --precision mixed --no-cpu-baseline --no-exact-compare --steps 5 --warmup 2 > $OUT/c5.json 2> $OUT/c5.err || exit 1
python3 $GRAFT_REPO_ROOT/tools/prof_stats.py $OUT/c5 40 | grep -i "cgemm\|coeffs"
python3 -c "import json; d=json.load(open('$OUT/c5.json')); k=d['kernels_ms_per_step']; print('C5', d['ms_per_step'], 'dft', k['grid_dft_fwd'], k['grid_dft_inv'])"

cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_grid.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > gpurun_out/exp_spread_tests.log 2>&1 && CF_EXP_SPREAD_PASS=32 timeout -k 10 300 python -u -m pytest tests/test_gpu_grid.py -x -q --timeout 200 --timeout-method thread >> gpurun_out/exp_spread_tests.log 2>&1 && bash tools/exp_spread2.sh

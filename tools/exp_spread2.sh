cd $GRAFT_REPO_ROOT
B="python -u bench.py --no-cpu-baseline --no-exact-compare --steps 20 --warmup 5"
for cfg in "CF_EXP_SPREAD_PASS=32" "CF_EXP_SPREAD_PASS=64"; do
  env $cfg timeout -k 10 120 $B > gpurun_out/sp_tmp.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/sp_tmp.json')); k=d['kernels_ms_per_step']; print('$cfg', d['ms_per_step'], k['grid_spread'])" >> gpurun_out/exp_spread2.txt
done

cd $GRAFT_REPO_ROOT
B="python -u bench.py --no-cpu-baseline --no-exact-compare --steps 20 --warmup 5"
for cfg in "" "CF_EXP_NO_EG=1" "CF_EXP_NO_LJFIRST=1" "CF_EXP_NO_EG=1 CF_EXP_NO_LJFIRST=1"; do
  echo "== $cfg" >> gpurun_out/exp1.txt
  env $cfg timeout -k 10 120 $B > gpurun_out/exp1_tmp.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/exp1_tmp.json')); print(d['ms_per_step'], d['kernels_ms_per_step']['direct_pairs'], d['kernels_ms_per_step']['neighbor_list'])" >> gpurun_out/exp1.txt
done

cd $GRAFT_REPO_ROOT
B="python -u bench.py --no-cpu-baseline --no-exact-compare --steps 40 --warmup 5"
for sk in 0.05 0.1 0.15 0.2 0.3; do
  timeout -k 10 120 $B --neighbor-skin $sk > gpurun_out/skin_tmp.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/skin_tmp.json')); k=d['kernels_ms_per_step']; print('$sk', d['ms_per_step'], k['direct_pairs'], k['neighbor_list'], k['cell_sort'], d['config']['nlist_builds_in_timed_steps'])" >> gpurun_out/exp_skin.txt
done

# GPU box: FETCH_SIZE / WRITE_SIZE passes (separate) for the grid spread and interpolation
set -e
cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/pmc_sf gpurun_out/pmc_sw
bash tools/pmc_one.sh sf "k_g_spread|k_g_interp" FETCH_SIZE
bash tools/pmc_one.sh sw "k_g_spread|k_g_interp" WRITE_SIZE
for x in sf sw; do python3 tools/pmc_show.py gpurun_out/pmc_$x; done > gpurun_out/pmc_spread.txt

set -e
cd $GRAFT_REPO_ROOT
bash tools/pmc_one.sh ga "k_g_spread|k_g_interp|k_g_cgemm" SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS
bash tools/pmc_one.sh gb "k_g_spread|k_g_interp|k_g_cgemm" SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE
bash tools/pmc_one.sh gc "k_g_spread|k_g_interp|k_g_cgemm" FETCH_SIZE
bash tools/pmc_one.sh gd "k_g_spread|k_g_interp|k_g_cgemm" TA_BUSY_avr TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum
for x in ga gb gc gd; do python3 tools/pmc_show.py gpurun_out/pmc_$x; done > gpurun_out/pmc_grid.txt

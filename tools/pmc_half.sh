set -e
cd $GRAFT_REPO_ROOT
bash tools/pmc_one.sh ha "k_pairs" SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS
bash tools/pmc_one.sh hb "k_pairs" SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE SQ_WAVES
bash tools/pmc_one.sh hc "k_pairs" TA_BUSY_avr TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum
for x in ha hb hc; do python3 tools/pmc_show.py gpurun_out/pmc_$x; done > gpurun_out/pmc_half.txt

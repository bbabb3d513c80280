set -e
cd $GRAFT_REPO_ROOT
bash tools/pmc_one.sh na "k_nlist" SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS
bash tools/pmc_one.sh nb "k_nlist" SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_BRANCH GRBM_GUI_ACTIVE
bash tools/pmc_one.sh nc "k_nlist" WRITE_SIZE
bash tools/pmc_one.sh nd "k_nlist" FETCH_SIZE
for x in na nb nc nd; do python3 tools/pmc_show.py gpurun_out/pmc_$x; done > gpurun_out/pmc_nlist.txt

set -e
cd $GRAFT_REPO_ROOT
bash tools/pmc_one.sh pa "k_pairs" SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS
bash tools/pmc_one.sh pb "k_pairs" SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE
bash tools/pmc_one.sh pc "k_pairs" TA_BUSY_avr TA_BUSY_max TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum
python3 tools/pmc_show.py gpurun_out/pmc_pa > gpurun_out/pmc_pairs.txt
python3 tools/pmc_show.py gpurun_out/pmc_pb >> gpurun_out/pmc_pairs.txt
python3 tools/pmc_show.py gpurun_out/pmc_pc >> gpurun_out/pmc_pairs.txt

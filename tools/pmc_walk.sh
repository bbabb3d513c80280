# GPU box: PMC passes over k_pairs_half, two-pass walk (CF_PAIRWALK=1) vs one pass (0)
set -e
cd $GRAFT_REPO_ROOT
for w in 1 0; do
  export CF_PAIRWALK=$w
  bash tools/pmc_one.sh w${w}a "k_pairs_half" SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD
  bash tools/pmc_one.sh w${w}b "k_pairs_half" FETCH_SIZE GRBM_GUI_ACTIVE SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS
  bash tools/pmc_one.sh w${w}c "k_pairs_half" TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TA_BUSY_avr TCC_HIT_sum
done
for x in w1a w1b w1c w0a w0b w0c; do echo "== $x"; python3 tools/pmc_show.py gpurun_out/pmc_$x; done > gpurun_out/pmc_walk.txt
cat gpurun_out/pmc_walk.txt

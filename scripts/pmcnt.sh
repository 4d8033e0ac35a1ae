set -o pipefail
export PMC_GROUPS="FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum;SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE;TA_BUSY_avr TA_TA_BUSY_sum"
bash scripts/pmc_workload.sh pmcnt sdd16k_nt "--workload op --op sdd --trans NT --density 0.5 --k 16384" || exit 1
bash scripts/pmc_workload.sh pmcnt sdd16k_nn "--workload op --op sdd --trans NN --density 0.5 --k 16384" || exit 1
bash scripts/pmc_workload.sh pmcnt sdd16k_tt "--workload op --op sdd --trans TT --density 0.5 --k 16384" || exit 1

set -o pipefail
export SPUTNIK_AMD_GROUPED_MIN_PER_CU=4
export PMC_GROUPS="FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum;SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE;TA_BUSY_avr TA_TA_BUSY_sum;TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"
bash scripts/pmc_workload.sh pmcx sdd4096 "--workload op --op sdd --trans NN --density 1.0 --k 4096" || exit 1
bash scripts/pmc_workload.sh pmcx dsd4096 "--workload op --op dsd --trans NN --density 1.0 --k 4096" || exit 1

set -o pipefail
export PMC_GROUPS="FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum;SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE;TA_BUSY_avr TA_TA_BUSY_sum;TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum;TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum"
A="--workload op --op sdd --trans NN --density 0.5 --k 16384"
SPUTNIK_AMD_SDD4W_MAX_LD=16384 bash scripts/pmc_workload.sh pmc16k sdd16k_w8 "$A" || exit 1
SPUTNIK_AMD_SDD4W_MAX_LD=32768 bash scripts/pmc_workload.sh pmc16k sdd16k_w4 "$A" || exit 1
A="--workload op --op sdd --trans NN --density 0.5 --k 15872"
SPUTNIK_AMD_SDD4W_MAX_LD=32768 bash scripts/pmc_workload.sh pmc16k sdd15872_w4 "$A" || exit 1
SPUTNIK_AMD_GROUPED_SDD=0 bash scripts/pmc_workload.sh pmc16k sdd15872_w8 "$A" || exit 1

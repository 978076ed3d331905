set -u
mkdir -p gpurun_out/pmc_mn
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
i=0
for ctrs in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS" "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "TA_BUSY_avr TA_TA_BUSY_sum" "GRBM_GUI_ACTIVE SQ_INSTS_VMEM"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $ctrs -d gpurun_out/pmc_mn/p$i -o run --output-format csv -- python tools/gemm_pmc_one.py > gpurun_out/pmc_mn/p$i.log 2>&1 || exit 1
done

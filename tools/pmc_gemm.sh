# PMC passes over tools/gemm_one.py (one rocprofv3 run per counter set) + summary
set -u
export TMPDIR=/tmp
shape=${1:-fc1f}
O=gpurun_out/pmc_gemm_$shape
mkdir -p $O
i=0
for ctrs in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS" \
            "SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_VMEM" \
            "TA_BUSY_avr TA_TA_BUSY_sum GRBM_GUI_ACTIVE" ; do
  i=$((i+1))
  GEMM_ONE=$shape timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $ctrs -d $O/p$i -o run --output-format csv -- \
    python tools/gemm_one.py > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
python tools/pmc_summary.py $O gemm_bf16

set -u
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT -d gpurun_out/pmc/p1 -o run --output-format csv -- python tools/gemm_one.py > gpurun_out/pmc/p1.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc/p2 -o run --output-format csv -- python tools/gemm_one.py > gpurun_out/pmc/p2.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/pmc/p3 -o run --output-format csv -- python tools/gemm_one.py > gpurun_out/pmc/p3.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE GRBM_GUI_ACTIVE -d gpurun_out/pmc/p4 -o run --output-format csv -- python tools/gemm_one.py > gpurun_out/pmc/p4.log 2>&1 || exit 1

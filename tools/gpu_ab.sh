# same-box A/B: working tree (A) vs ab/base build (B): GEMM microbench + bench
set -u
mkdir -p gpurun_out/ab
rm -f gpurun_out/ab/summary.txt
timeout -k 10 200 python tools/gemm_vs_blas.py > gpurun_out/ab/gemm_A.log 2>&1 || exit 1
CG_LIB_PATH=ab/base/libcodonlm_hip.so timeout -k 10 200 python tools/gemm_vs_blas.py > gpurun_out/ab/gemm_B.log 2>&1 || exit 1
bash tools/ab.sh "CG_X=1" "CG_LIB_PATH=ab/base/libcodonlm_hip.so" ${REPS:-2}

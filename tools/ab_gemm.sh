# GEMM change gate: GEMM op tests, then same-box A/B of the bench vs ab/base
set -u
mkdir -p gpurun_out/ab
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -x -q -k "gemm" -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/ab/pytest.log 2>&1 || exit 1
timeout -k 10 200 python tools/dw_sweep.py > gpurun_out/ab/dw_A.log 2>&1 || exit 1
CG_LIB_PATH=ab/base/libcodonlm_hip.so timeout -k 10 200 python tools/dw_sweep.py > gpurun_out/ab/dw_B.log 2>&1 || exit 1
rm -f gpurun_out/ab/summary.txt
bash tools/ab.sh "CG_X=1" "CG_LIB_PATH=ab/base/libcodonlm_hip.so" 2

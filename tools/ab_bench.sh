# same-box A/B of the bench: working tree (A) vs ab/base (B), after the op + model GPU tests
set -u
mkdir -p gpurun_out/ab
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py tests/test_gpu_aux.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/ab/pytest.log 2>&1 || { tail -30 gpurun_out/ab/pytest.log; exit 1; }
tail -1 gpurun_out/ab/pytest.log
rm -f gpurun_out/ab/summary.txt
bash tools/ab.sh "CG_X=1" "CG_LIB_PATH=ab/base/libcodonlm_hip.so" ${REPS:-2}

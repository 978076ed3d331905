set -u
mkdir -p gpurun_out/ab
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -m gpu -x -q -k "attn or dropout" -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/ab/pytest.log 2>&1 || exit 1
rm -f gpurun_out/ab/summary.txt
bash tools/ab.sh "CG_X=1" "CG_LIB_PATH=ab/base/libcodonlm_hip.so" 2

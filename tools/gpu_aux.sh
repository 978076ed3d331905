set -u
mkdir -p gpurun_out/aux
timeout -k 10 300 python -u -m pytest tests/test_gpu_aux.py tests/test_gpu_model.py -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/aux/pytest.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/aux/pytest.log; exit $rc

# KV-cache decode GPU tests
set -u
mkdir -p gpurun_out/decode
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_inference.py -m gpu -x -v -p no:cacheprovider --timeout 180 --timeout-method thread > gpurun_out/decode/pytest.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/decode/pytest.log; exit $rc

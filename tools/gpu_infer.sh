# inference GPU tests (pooling kernel, extract_embeddings / query_model CLIs)
set -u
mkdir -p gpurun_out/infer
timeout -k 10 400 python -u -m pytest tests/test_gpu_inference.py -m gpu -x -v -p no:cacheprovider --timeout 180 --timeout-method thread > gpurun_out/infer/pytest.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/infer/pytest.log; exit $rc

# trainer GPU tests (device batches, nonfinite/resume counters, end-to-end aux run)
set -u
mkdir -p gpurun_out/train
timeout -k 10 400 python -u -m pytest tests/test_gpu_training.py -m gpu -x -v -p no:cacheprovider --timeout 180 --timeout-method thread > gpurun_out/train/pytest.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/train/pytest.log; exit $rc

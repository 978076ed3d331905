set -u
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_ops.py -q -p no:cacheprovider --timeout=300 -x -k "gemm" > gpurun_out/pytest_gemm.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gemm.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/ref_cmp.py > gpurun_out/ref_cmp.log 2>&1 || exit 1
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1
echo "bench rc=$?" >> gpurun_out/bench.log

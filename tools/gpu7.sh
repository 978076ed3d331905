set -u
mkdir -p gpurun_out/prof5
timeout -k 10 300 python -m pytest tests/test_gpu_model.py -q -p no:cacheprovider --timeout=300 -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1
echo "bench rc=$?" >> gpurun_out/bench.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof5 -o run --output-format csv -- python bench.py --no-cpu-baseline > gpurun_out/prof5/bench.log 2>&1
echo "prof rc=$?" >> gpurun_out/prof5/bench.log

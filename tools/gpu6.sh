set -u
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout=300 -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
mkdir -p gpurun_out/prof4
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof4 -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-roofline > gpurun_out/prof4/bench.log 2>&1
echo "prof rc=$?" >> gpurun_out/prof4/bench.log

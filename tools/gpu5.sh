set -u
mkdir -p gpurun_out/prof3
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof3 -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-roofline > gpurun_out/prof3/bench.log 2>&1
echo "prof rc=$?" >> gpurun_out/prof3/bench.log

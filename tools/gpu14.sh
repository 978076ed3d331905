set -u
mkdir -p gpurun_out/prof14
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof14 -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-kernel-roofline > gpurun_out/prof14/bench.log 2>&1 || exit 1
f=$(find gpurun_out/prof14 -name "*kernel_stats.csv" | head -1)
python tools/kstats.py "$f" 13 40 > gpurun_out/prof14/kstats.txt

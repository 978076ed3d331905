set -u
O=gpurun_out/c5
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --steps 10 --warmup 3 > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python bench.py --config c5 --no-cpu-baseline --no-kernel-roofline --steps 10 --warmup 3 > $O/trace.log 2>&1 || exit 1

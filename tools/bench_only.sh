set -u
mkdir -p gpurun_out/round
timeout -k 10 300 python bench.py > gpurun_out/round/bench.json 2> gpurun_out/round/bench.err || exit 1

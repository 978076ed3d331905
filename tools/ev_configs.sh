set -u
mkdir -p gpurun_out/ev
for c in c2 c3 c5; do
  timeout -k 10 300 python bench.py --config $c > gpurun_out/ev/bench_$c.json 2> gpurun_out/ev/bench_$c.err || exit 1
  cat gpurun_out/ev/bench_$c.json
done

# Bench lines of the other BASELINE configs (C2, C3, C5) and the C4 trainer path, one box, with the
# CPU baseline off (it is the same oracle trainer as the C4 line's) -> gpurun_out/ev/
set -u
mkdir -p gpurun_out/ev
for c in c2 c3 c5; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > gpurun_out/ev/bench_$c.json 2> gpurun_out/ev/bench_$c.err || exit 1
  cat gpurun_out/ev/bench_$c.json
done
timeout -k 10 300 python bench.py --path trainer --no-cpu-baseline > gpurun_out/ev/bench_c4_trainer.json 2> gpurun_out/ev/bench_c4_trainer.err || exit 1
cat gpurun_out/ev/bench_c4_trainer.json

# rocprofv3 kernel-trace summary of the bench (no probe passes: exactly warmup+steps steps)
set -u
mkdir -p gpurun_out/prof_step
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_step -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-roofline ${BENCH_ARGS:-} > gpurun_out/prof_step/bench.log 2>&1
echo "rc=$?" >> gpurun_out/prof_step/bench.log

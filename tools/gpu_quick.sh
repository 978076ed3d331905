# quick GPU gate: parity tests + one bench line (no cpu baseline)
set -u
mkdir -p gpurun_out/quick
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/quick/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/quick/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/quick/bench.log 2>&1 || exit 1

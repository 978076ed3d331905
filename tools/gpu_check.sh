# GPU check: parity tests, bench line, rocprof kernel-trace summary (one gpurun call)
set -u
mkdir -p gpurun_out/check
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/check/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/check/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python __graft_entry__.py > gpurun_out/check/smoke.log 2>&1 || exit 1
timeout -k 10 400 python bench.py > gpurun_out/check/bench.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/check/prof -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/check/bench_prof.log 2>&1
echo "prof rc=$?" >> gpurun_out/check/bench_prof.log

# round evidence: rocprofv3 kernel-trace stats of the bench command, HBM PMC passes
# (FETCH_SIZE / WRITE_SIZE in separate runs), then the bench line itself (with cpu_baseline)
set -u
OUT=gpurun_out/round
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python bench.py --no-cpu-baseline > $OUT/trace_bench.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-kernel-roofline > $OUT/pmc_fetch.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-kernel-roofline > $OUT/pmc_write.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1

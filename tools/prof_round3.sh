# Round evidence (rounds 3, 4) for one config: a bench line (with the live roofline probe), the rocprofv3
# kernel-trace stats of the bench command, the HBM PMC passes (FETCH_SIZE / WRITE_SIZE in separate
# runs) and the kernel summary per step.
#   [ROUND=r4] bash tools/prof_round3.sh c4 [extra bench args]    -> gpurun_out/${ROUND:-r3}_<cfg>/
set -u
cfg=${1:-c4}; shift || true
O=gpurun_out/${ROUND:-r3}_$cfg
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --config $cfg "$@" > $O/bench.json 2> $O/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
  python bench.py --config $cfg --no-cpu-baseline --no-kernel-roofline --steps 20 --warmup 5 "$@" > $O/trace.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- \
  python bench.py --config $cfg --steps 3 --warmup 2 --no-cpu-baseline --no-kernel-roofline "$@" > $O/pmc_fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- \
  python bench.py --config $cfg --steps 3 --warmup 2 --no-cpu-baseline --no-kernel-roofline "$@" > $O/pmc_write.log 2>&1
rc=$?
f=$(find $O/trace -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && python tools/kstats.py "$f" 25 40 > $O/kernel_stats_per_step.txt
exit $rc

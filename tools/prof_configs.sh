# Per-config evidence: one bench line (kernel roofline, no CPU leg) and the rocprofv3 kernel-trace
# stats of the same command, for each config given (default: c2 c3 c5 c4).
#   bash tools/prof_configs.sh [cfg ...]   -> gpurun_out/cfg_<cfg>/{bench.json,trace/,kernel_stats_per_step.txt}
set -u
export TMPDIR=/tmp
cfgs=${*:-c2 c3 c5 c4}
for cfg in $cfgs; do
  O=gpurun_out/cfg_$cfg
  mkdir -p $O
  timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
    python bench.py --config $cfg --no-cpu-baseline --no-kernel-roofline --steps 20 --warmup 5 > $O/trace.log 2>&1 || exit 1
  f=$(find $O/trace -name "*kernel_stats.csv" | head -1)
  python tools/kstats.py "$f" 25 30 > $O/kernel_stats_per_step.txt
  echo "$cfg $(head -c 300 $O/bench.json)"
done

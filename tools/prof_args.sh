# rocprofv3 kernel table of one bench.py argument set (C4 bench step, 20 steps after 5 warm-up):
#   bash tools/prof_args.sh <tag> [bench args]    -> gpurun_out/profargs_<tag>/
set -u
tag=$1; shift
export TMPDIR=/tmp
O=gpurun_out/profargs_$tag; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O -o run --output-format csv -- python bench.py --no-cpu-baseline --no-kernel-roofline --steps 20 --warmup 5 "$@" > $O/bench.log 2>&1 || exit 1
python tools/kstats.py $(ls $O/run_kernel_stats.csv $O/*/run_kernel_stats.csv 2>/dev/null | head -1) 25 16

# rocprofv3 kernel tables of two library builds on the same box (C4 bench step, 20 steps after 5
# warm-up each): the tree's own library and another build (tools/build_variant.sh, or a build of an
# earlier commit's sources) -> gpurun_out/r6prof_{base,new}/, printed per step.
#   bash tools/prof_lib_ab.sh var/base/libcodonlm_hip.so [bench args]
set -u
BASE=$1; shift
export TMPDIR=/tmp
for v in base new; do
  O=gpurun_out/r6prof_$v; mkdir -p $O
  if [ $v = base ]; then export CG_LIB_PATH=$BASE; else unset CG_LIB_PATH; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O -o run --output-format csv -- python bench.py --no-cpu-baseline --no-kernel-roofline --steps 20 --warmup 5 "$@" > $O/bench.log 2>&1 || exit 1
done
unset CG_LIB_PATH
for v in base new; do echo "== $v"; python tools/kstats.py $(ls gpurun_out/r6prof_$v/run_kernel_stats.csv gpurun_out/r6prof_$v/*/run_kernel_stats.csv 2>/dev/null | head -1) 25 12; done

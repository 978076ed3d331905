# One entry point for GPU-box work (run as: gpurun -- 'bash tools/gpu.sh <cmd> [args]').
# Every GPU step has its own time limit and the steps chain with && (a failure ends the call).
#
#   test  [pytest -k expr]      GPU tests (tests -m gpu), one process      -> gpurun_out/test/
#   full                        round-end gate: all GPU tests, then smoke() -> gpurun_out/full/
#   bench [bench.py args]       one bench line                               -> gpurun_out/bench/
#   prof  [tag] [bench args]    rocprofv3 --kernel-trace --stats of bench.py -> gpurun_out/prof_<tag>/
#   attn  [tag]                 rocprofv3 --kernel-trace --stats of tools/attn_one.py -> gpurun_out/attn_<tag>/
#   kprof <tag> <script> [args]  rocprofv3 --kernel-trace --stats of python <script> -> gpurun_out/kprof_<tag>/
#   pmc   <tag> <script> "<counter set>" ["<counter set>" ...]
#                               one rocprofv3 --pmc pass per counter set over python <script>
#                                                                            -> gpurun_out/pmc_<tag>/
set -u
cmd=${1:-test}
shift || true
export TMPDIR=/tmp
PYT="python -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread"
case "$cmd" in
  test)
    mkdir -p gpurun_out/test
    if [ $# -gt 0 ]; then k=(-k "$1"); else k=(); fi
    timeout -k 10 900 $PYT tests -m gpu -x -q "${k[@]}" > gpurun_out/test/pytest.log 2>&1
    rc=$?; tail -5 gpurun_out/test/pytest.log; exit $rc ;;
  full)
    mkdir -p gpurun_out/full
    timeout -k 10 900 $PYT tests -m gpu -x -q > gpurun_out/full/pytest.log 2>&1 &&
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/full/smoke.log 2>&1
    rc=$?; tail -3 gpurun_out/full/pytest.log; exit $rc ;;
  bench)
    mkdir -p gpurun_out/bench
    timeout -k 10 600 python bench.py "$@" > gpurun_out/bench/bench.json 2> gpurun_out/bench/bench.err
    rc=$?; cat gpurun_out/bench/bench.json; exit $rc ;;
  prof)
    tag=${1:-step}; shift || true
    O=gpurun_out/prof_$tag
    mkdir -p $O
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O -o run --output-format csv -- \
      python bench.py --no-cpu-baseline --no-kernel-roofline "$@" > $O/bench.log 2>&1
    rc=$?; tail -2 $O/bench.log; exit $rc ;;
  attn)
    tag=${1:-x}
    O=gpurun_out/attn_$tag
    mkdir -p $O
    timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O -o run --output-format csv -- \
      python tools/attn_one.py > $O/run.log 2>&1
    rc=$?; python tools/kstats.py $O/run_kernel_stats.csv 4 8; exit $rc ;;
  kprof)
    tag=$1; shift
    O=gpurun_out/kprof_$tag
    mkdir -p $O
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O -o run --output-format csv -- \
      python "$@" > $O/run.log 2>&1
    rc=$?; tail -3 $O/run.log; exit $rc ;;
  pmc)
    tag=$1; script=$2; shift 2
    O=gpurun_out/pmc_$tag
    mkdir -p $O
    i=0
    for ctrs in "$@"; do
      i=$((i+1))
      timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $ctrs -d $O/p$i -o run --output-format csv -- \
        python $script > $O/p$i.log 2>&1 || exit 1
    done ;;
  *)
    echo "unknown command $cmd"; exit 2 ;;
esac

# One GPU call for a library change: the GPU tests selected by a pytest -k expression, then a
# same-box interleaved A/B of the tree's library against another build on the given configs.
#   bash tools/gpu_ab_check.sh "<pytest -k expr>" <other lib> "c4 c5" [rounds]
set -u
K=$1; BASE=$2; CFGS=$3; R=${4:-2}
export TMPDIR=/tmp
mkdir -p gpurun_out/abcheck
timeout -k 10 700 python -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread tests -m gpu -x -q -k "$K" > gpurun_out/abcheck/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/abcheck/pytest.log; [ $rc -eq 0 ] || exit $rc
for c in $CFGS; do
  rm -f gpurun_out/ablib/summary.txt
  bash tools/ab_lib.sh "$BASE default" $R --config $c --steps 20 > /dev/null || exit 1
  echo "== $c"; cat gpurun_out/ablib/summary.txt
done

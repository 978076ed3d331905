# Same-box interleaved comparison of this tree's C4 bench step against another tree's (e.g. an
# earlier round's final commit, built under var/):   bash tools/ab_trees.sh var/r5tree [rounds] [bench args]
set -u
OTHER=$1; R=${2:-3}; shift 2 || true
export TMPDIR=/tmp
mkdir -p gpurun_out/abtrees
rm -f gpurun_out/abtrees/summary.txt
for r in $(seq 1 $R); do
  for v in other this; do
    if [ $v = other ]; then d=$OTHER; else d=.; fi
    (cd $d && timeout -k 10 300 python bench.py --no-cpu-baseline --no-kernel-roofline --steps 30 "$@") > gpurun_out/abtrees/$v$r.log 2>&1 || exit 1
    echo "$v r$r $(python -c "import json;d=json.loads(open('gpurun_out/abtrees/$v$r.log').read().strip().split(chr(10))[-1]);print(d['value'],d['ms_per_step'])")" >> gpurun_out/abtrees/summary.txt
  done
done
cat gpurun_out/abtrees/summary.txt

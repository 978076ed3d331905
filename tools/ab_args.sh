# Same-box interleaved A/B of two bench.py argument sets (same library):
#   bash tools/ab_args.sh "<args A>" "<args B>" [rounds]
set -u
mkdir -p gpurun_out/abargs
rm -f gpurun_out/abargs/summary.txt
R=${3:-3}
for r in $(seq 1 $R); do
  for v in A B; do
    if [ $v = A ]; then a="$1"; else a="$2"; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-kernel-roofline --steps 30 $a > gpurun_out/abargs/$v$r.log 2>&1 || exit 1
    echo "$v [$a] $(python -c "import json;d=json.loads(open('gpurun_out/abargs/$v$r.log').read().strip().split(chr(10))[-1]);print(d['value'],d['ms_per_step'])")" >> gpurun_out/abargs/summary.txt
  done
done
cat gpurun_out/abargs/summary.txt

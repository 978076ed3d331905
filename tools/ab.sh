# A/B of two environment settings on the same box: bash tools/ab.sh "ENV_A" "ENV_B" [reps]
set -u
mkdir -p gpurun_out/ab
reps=${3:-2}
for r in $(seq 1 $reps); do
  for v in A B; do
    if [ $v = A ]; then e="$1"; else e="$2"; fi
    env $e timeout -k 10 300 python bench.py --no-cpu-baseline --no-kernel-roofline --steps 30 > gpurun_out/ab/$v$r.log 2>&1 || exit 1
    echo "$v [$e] $(python -c "import json,sys;d=json.loads(open('gpurun_out/ab/$v$r.log').read().strip().split(chr(10))[-1]);print(d['value'],d['ms_per_step'])")" >> gpurun_out/ab/summary.txt
  done
done
cat gpurun_out/ab/summary.txt

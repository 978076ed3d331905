# Same-box A/B of library builds on the full C4 bench step (interleaved, `reps` rounds):
#   bash tools/ab_lib.sh "<lib path or 'default'> ..." [reps] [bench args]
set -u
mkdir -p gpurun_out/ablib
libs=$1; reps=${2:-2}; shift 2 || true
for r in $(seq 1 $reps); do
  for lib in $libs; do
    tag=$(echo $lib | tr '/' '_')
    if [ "$lib" = default ]; then e=""; else e="CG_LIB_PATH=$lib"; fi
    env $e timeout -k 10 300 python bench.py --no-cpu-baseline --no-kernel-roofline --steps 30 "$@" > gpurun_out/ablib/$tag.$r.log 2>&1 || exit 1
    echo "$lib r$r $(python -c "import json;d=json.loads(open('gpurun_out/ablib/$tag.$r.log').read().strip().split(chr(10))[-1]);print(d['value'],d['ms_per_step'])")" >> gpurun_out/ablib/summary.txt
  done
done
cat gpurun_out/ablib/summary.txt

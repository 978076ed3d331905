# Same-box A/B of library builds on several bench configs (interleaved, `reps` rounds):
#   bash tools/ab_lib_cfg.sh "<lib|default> ..." "<config> ..." [reps]
set -u
mkdir -p gpurun_out/ablibc
libs=$1; cfgs=$2; reps=${3:-2}
for r in $(seq 1 $reps); do
  for c in $cfgs; do
    for lib in $libs; do
      tag=$(echo $lib | tr '/' '_')
      if [ "$lib" = default ]; then e=""; else e="CG_LIB_PATH=$lib"; fi
      env $e timeout -k 10 300 python bench.py --no-cpu-baseline --no-kernel-roofline --steps 30 --config $c > gpurun_out/ablibc/$c.$tag.$r.log 2>&1 || exit 1
      echo "$c $lib r$r $(python -c "import json;d=json.loads(open('gpurun_out/ablibc/$c.$tag.$r.log').read().strip().split(chr(10))[-1]);print(d['value'],d['ms_per_step'])")" >> gpurun_out/ablibc/summary.txt
    done
  done
done
cat gpurun_out/ablibc/summary.txt

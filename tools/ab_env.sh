# Interleaved same-box A/B of bench.py under two environment settings (extra bench args after --):
#   bash tools/ab_env.sh <reps> "ENV_A" "ENV_B" [bench args]
set -u
reps=$1; a=$2; b=$3; shift 3
O=gpurun_out/ab_env
mkdir -p $O
for r in $(seq 1 $reps); do
  for v in A B; do
    if [ $v = A ]; then e="$a"; else e="$b"; fi
    env $e timeout -k 10 300 python bench.py --no-cpu-baseline --no-kernel-roofline --steps 30 "$@" > $O/$v$r.json 2> $O/$v$r.err || exit 1
    echo "$v [$e] $(grep -o '"ms_per_step": [0-9.]*' $O/$v$r.json)" >> $O/summary.txt
  done
done
cat $O/summary.txt

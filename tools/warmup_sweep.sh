set -u
O=gpurun_out/warmup; mkdir -p $O
for r in 1 2 3; do
  for a in "--steps 20 --warmup 5" "--steps 20 --warmup 40" "--steps 100 --warmup 5"; do
    ms=$(timeout -k 10 120 python bench.py $a --no-cpu-baseline --no-kernel-roofline 2>/dev/null | python -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])") || exit 1
    echo "round $r [$a] $ms" | tee -a $O/out.txt
  done
done

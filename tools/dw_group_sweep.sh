# dW group-size / tile sweep of the bf16 engine per config (bench.py ms/step; same box, interleaved)
#   bash tools/dw_group_sweep.sh c3 "0 2 3 4 5 10" "0 128 256"
set -u
cfg=$1; groups=$2; tiles=${3:-0}
O=gpurun_out/dwsweep_$cfg; mkdir -p $O
for r in 1 2; do
  for g in $groups; do
    for t in $tiles; do
      env_g=""; env_t=""
      [ "$g" != 0 ] && env_g="CG_DW_GROUP=$g"
      [ "$t" != 0 ] && env_t="CG_DW_BM=$t"
      ms=$(env $env_g $env_t timeout -k 10 120 python bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-roofline 2>/dev/null | python -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])") || exit 1
      echo "round $r group $g tile $t ms_per_step $ms" | tee -a $O/out.txt
    done
  done
done

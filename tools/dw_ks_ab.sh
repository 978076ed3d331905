# grouped-dW token-range split A/B: planner's choice (auto) vs no split (CG_DW_KSPLIT=1), interleaved
#   bash tools/dw_ks_ab.sh "c2 c3 c5 c4"
set -u
cfgs=${1:-"c2 c3 c5 c4"}
O=gpurun_out/dw_ks_ab; mkdir -p $O
for r in 1 2; do
  for cfg in $cfgs; do
    for ks in 1 auto; do
      env_k=""; [ "$ks" != auto ] && env_k="CG_DW_KSPLIT=$ks"
      ms=$(env $env_k timeout -k 10 180 python bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-roofline 2>/dev/null | python -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])") || exit 1
      echo "round $r cfg $cfg ks $ks ms_per_step $ms" | tee -a $O/out.txt
    done
  done
done

# Same-box sweep of library switches on one config: bench.py ms/step, interleaved rounds
#   bash tools/env_sweep.sh c4 3 "" "CG_ATTN_FUSED_KEEP=0" ...
set -u
cfg=$1; rounds=$2; shift 2
O=gpurun_out/envsweep_$cfg; mkdir -p $O
for r in $(seq 1 $rounds); do
  for e in "$@"; do
    ms=$(env $e timeout -k 10 120 python bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-roofline 2>/dev/null | python -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])") || exit 1
    echo "round $r [${e:-default}] ms_per_step $ms" | tee -a $O/out.txt
  done
done

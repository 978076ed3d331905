# residual-prefetch A/B (CG_LW_RPF): per-product C4 GEMM times and the C4 step, default vs var/rpf1
set -u
O=gpurun_out/rpf; mkdir -p $O
for r in 1 2; do
  for v in "" var/rpf1/libcodonlm_hip.so; do
    echo "== lib ${v:-default} round $r" >> $O/out.txt
    CG_LIB_PATH=$v timeout -k 10 120 python tools/gemm_c4.py >> $O/out.txt 2>&1 || exit 1
    CG_LIB_PATH=$v timeout -k 10 180 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-roofline 2>/dev/null | python -c "import json,sys; print('ms_per_step', json.loads(sys.stdin.read())['ms_per_step'])" >> $O/out.txt || exit 1
  done
done

# Persistent-GEMM kernel choice per product: tools/gemm_c4.py under CG_PERS_LW = 0 (no loader
# waves), 1 (loader waves for plain / bias products: the default), 2 (loader waves for every
# epilogue), interleaved over rounds.   bash tools/gemm_lwmode.sh <rounds>
set -u
O=gpurun_out/gemm_lwmode
mkdir -p $O
for r in $(seq 1 ${1:-2}); do
  for m in 0 1 2; do
    echo "== round $r CG_PERS_LW=$m" >> $O/summary.txt
    CG_PERS_LW=$m timeout -k 10 200 python tools/gemm_c4.py >> $O/summary.txt 2>&1 || exit 1
  done
done
cat $O/summary.txt

# Same-box A/B of the C4 persistent-GEMM products (tools/gemm_c4.py) for two or more builds,
# interleaved over rounds.   bash tools/gemm_ab.sh <rounds> lib1.so lib2.so ...
set -u
rounds=$1; shift
O=gpurun_out/gemm_ab
mkdir -p $O
for r in $(seq 1 $rounds); do
  i=0
  for lib in "$@"; do
    i=$((i+1))
    echo "== round $r lib $i $lib" >> $O/summary.txt
    CG_LIB_PATH=$lib timeout -k 10 200 python tools/gemm_c4.py "${GEMM_ROWS:-}" >> $O/summary.txt 2>&1 || exit 1
  done
done
cat $O/summary.txt

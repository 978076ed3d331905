# colsum epilogue cost split (CG_COLSUM_DIAG builds: 1 no DPP sums, 2 no partial stores, 3 no accumulation)
set -u
O=gpurun_out/csd; mkdir -p $O
for r in 1 2; do
  for v in "" var/csd1/libcodonlm_hip.so var/csd2/libcodonlm_hip.so var/csd3/libcodonlm_hip.so; do
    echo "== lib ${v:-default} round $r" >> $O/out.txt
    CG_LIB_PATH=$v timeout -k 10 120 python tools/gemm_c4.py 2>&1 | grep "fc2 dX" >> $O/out.txt || exit 1
  done
done

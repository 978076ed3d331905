set -u
O=gpurun_out/pf; mkdir -p $O
for r in 1 2; do
  for v in "" var/pf1/libcodonlm_hip.so var/pf2/libcodonlm_hip.so var/pf4/libcodonlm_hip.so; do
    echo "== lib ${v:-default} round $r" >> $O/out.txt
    CG_LIB_PATH=$v timeout -k 10 120 python tools/gemm_c4.py >> $O/out.txt 2>&1 || exit 1
  done
done

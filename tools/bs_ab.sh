set -u
O=gpurun_out/bs; mkdir -p $O
CG_LIB_PATH=var/bs1/libcodonlm_hip.so timeout -k 10 600 python -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_ops.py -x -q -k "gemm" > $O/test.log 2>&1 || { tail -20 $O/test.log; exit 1; }
tail -2 $O/test.log
for r in 1 2; do
  for v in "" var/bs1/libcodonlm_hip.so; do
    echo "== lib ${v:-default} round $r" >> $O/out.txt
    CG_LIB_PATH=$v timeout -k 10 120 python tools/gemm_c4.py >> $O/out.txt 2>&1 || exit 1
  done
done

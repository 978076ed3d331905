set -u
O=gpurun_out/f32ab; mkdir -p $O
CG_LIB_PATH=var/bk32/libcodonlm_hip.so timeout -k 10 600 python -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_ops.py -x -q -k "gemm_layouts or gemm_epilogues or wide_tile" > $O/test.log 2>&1 || { tail -20 $O/test.log; exit 1; }
tail -1 $O/test.log
for r in 1 2; do
  for v in "" var/bk32/libcodonlm_hip.so; do
    echo "== lib ${v:-default} round $r" >> $O/out.txt
    CG_LIB_PATH=$v timeout -k 10 120 python tools/f32_gemm_time.py >> $O/out.txt 2>&1 || exit 1
  done
done

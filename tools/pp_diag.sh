set -u
O=gpurun_out/diag; mkdir -p $O
for r in 1 2; do
  CG_PERS_PP=0 timeout -k 10 120 python tools/gemm_diag.py >> $O/out.txt 2>&1 || exit 1
  for v in "" var/pp_d1/libcodonlm_hip.so var/pp_d2/libcodonlm_hip.so var/pp_d3/libcodonlm_hip.so; do
    if [ -n "$v" ]; then export CG_LIB_PATH=$v; else unset CG_LIB_PATH; fi
    echo "-- pp $v" >> $O/out.txt
    CG_PERS_PP=1 timeout -k 10 120 python tools/gemm_diag.py >> $O/out.txt 2>&1 || exit 1
  done
  unset CG_LIB_PATH
done
grep -v amdgpu.ids $O/out.txt

# SwiGLU-backward epilogue load pieces A/B (CG_DSW_NP builds), C3 products + C3 step
set -u
O=gpurun_out/dsw; mkdir -p $O
for r in 1 2; do
  for v in "" var/dswnp1/libcodonlm_hip.so var/dswnp2/libcodonlm_hip.so; do
    echo "== lib ${v:-default} round $r" >> $O/out.txt
    CG_LIB_PATH=$v timeout -k 10 120 python tools/gemm_c3_swiglu.py >> $O/out.txt 2>&1 || exit 1
  done
done

# Same-box A/B of library variants on the attention backward (tools/attn_bwd_ab.py, fused algo rows):
#   bash tools/attn_bwd_var.sh "<configs>" base var/<name> ...   (base = the in-tree build)
cfgs=$1; shift
for v in "$@" "$@"; do
  if [ "$v" = base ]; then unset CG_LIB_PATH; else export CG_LIB_PATH=$PWD/$v/libcodonlm_hip.so; fi
  echo "== $v"
  timeout -k 10 120 python -u tools/attn_bwd_ab.py $cfgs --rounds 1 2>&1 | grep '"algo"' || exit 1
done

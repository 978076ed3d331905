# attention-variant A/B plus the attention parity tests run against each variant build
set -u
bash tools/attn_ab.sh 2 genomics-lm_amd/codonlm_amd/libcodonlm_hip.so "$@" > /dev/null || exit 1
for v in "$@"; do
  echo "== tests $v" >> gpurun_out/attn_ab/tests.txt
  CG_LIB_PATH=$v timeout -k 10 300 python -u -m pytest -p no:cacheprovider --timeout 120 --timeout-method thread tests -m gpu -x -q -k "attention or attn" 2>&1 | tail -1 >> gpurun_out/attn_ab/tests.txt || exit 1
done

set -u
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout=300 -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python tools/attn_var.py > gpurun_out/attn_var.log 2>&1 || exit 1
CG_LIB_PATH=ab/base/libcodonlm_hip.so timeout -k 10 200 python tools/attn_var.py > gpurun_out/attn_var_base.log 2>&1 || exit 1
rm -f gpurun_out/ab/summary.txt
bash tools/ab.sh "CG_X=1" "CG_LIB_PATH=ab/base/libcodonlm_hip.so" 2 || exit 1
bash tools/pmc_attn.sh

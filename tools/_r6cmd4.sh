mkdir -p gpurun_out/r6cs && export TMPDIR=/tmp &&
timeout -k 10 600 python -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread tests -m gpu -x -q -k "dw_grouped or bf16_engine or dw_plan or bench_batch or c4_layer_grad or dropout_training" > gpurun_out/r6cs/pytest.log 2>&1 && tail -1 gpurun_out/r6cs/pytest.log &&
rm -f gpurun_out/ablib/summary.txt && bash tools/ab_lib.sh "var/base/libcodonlm_hip.so default" 3 --steps 30 && cp gpurun_out/ablib/summary.txt gpurun_out/r6cs/ab_c4_v2.txt &&
bash tools/_r6cmd3.sh

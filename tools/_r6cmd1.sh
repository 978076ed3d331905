mkdir -p gpurun_out/parity gpurun_out/r6ab && export TMPDIR=/tmp &&
timeout -k 10 800 python -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread tests -m gpu -x -v -s -k "fp32 or neartie or forced_tile or algo_errors or fused" > gpurun_out/parity/pytest.log 2>&1 && tail -3 gpurun_out/parity/pytest.log &&
for a in split fused split fused; do timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-roofline --attn-bwd $a >> gpurun_out/r6ab/c5.jsonl 2>>gpurun_out/r6ab/err.log || exit 1; done &&
timeout -k 10 400 python bench.py --config c4 --steps 20 --warmup 5 > gpurun_out/r6ab/c4.json 2>>gpurun_out/r6ab/err.log && cat gpurun_out/r6ab/c4.json

set -u
O=gpurun_out/c5
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_aux.py tests/test_gpu_training.py -m gpu -x -q -p no:cacheprovider --timeout 180 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --steps 10 --warmup 3 > $O/bench2.json 2> $O/bench2.err || exit 1

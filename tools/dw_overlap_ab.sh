# last-dW-group overlap A/B (CG_DW_OVERLAP): gradient tests, then interleaved steps on vs off
set -u
O=gpurun_out/dwov; mkdir -p $O
timeout -k 10 600 python -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread tests -m gpu -x -q -k "dw_plan or configs or c4_layer or trainer or aux" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2; do
  for cfg in c4 c3 c5 c2; do
    for ov in 1 0; do
      ms=$(CG_DW_OVERLAP=$ov timeout -k 10 180 python bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-roofline 2>/dev/null | python -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])") || exit 1
      echo "round $r cfg $cfg overlap $ov ms_per_step $ms" | tee -a $O/out.txt
    done
  done
done

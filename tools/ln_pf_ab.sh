# LayerNorm row-prefetch A/B: LN op + engine parity tests at the default (by-measurement) setting,
# then interleaved steps, default vs CG_LN_PF=0 (no prefetch)
set -u
O=gpurun_out/lnpf2; mkdir -p $O
timeout -k 10 600 python -u -m pytest -p no:cacheprovider --timeout 300 --timeout-method thread tests -m gpu -x -q -k "layernorm or ln_ or configs or c4_layer or hd48" > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2; do
  for cfg in c4 c3 c5; do
    for pf in default 0; do
      env_p=""; [ "$pf" != default ] && env_p="CG_LN_PF=$pf"
      ms=$(env $env_p timeout -k 10 180 python bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-roofline 2>/dev/null | python -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])") || exit 1
      echo "round $r cfg $cfg ln_pf $pf ms_per_step $ms" | tee -a $O/out.txt
    done
  done
done

# per-kernel LayerNorm times under each CG_LN_PF setting (rocprofv3 kernel stats of a C4 / C3 bench)
set -u
export TMPDIR=/tmp
for cfg in c4 c3; do
for pf in 0 1 2 3; do
  O=gpurun_out/lnpf_prof/${cfg}_$pf; mkdir -p $O
  CG_LN_PF=$pf timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O -o run --output-format csv -- \
    python bench.py --config $cfg --no-cpu-baseline --no-kernel-roofline --steps 20 --warmup 5 > $O/log.txt 2>&1 || exit 1
  f=$(find $O -name "*kernel_stats.csv" | head -1)
  echo "== $cfg CG_LN_PF=$pf" >> gpurun_out/lnpf_prof/summary.txt
  grep -E "ln_(fwd|bwd)" "$f" | cut -d, -f1-5 >> gpurun_out/lnpf_prof/summary.txt
done
done

# Same-box per-kernel A/B of attention builds: rocprofv3 --kernel-trace --stats of tools/attn_time.py
# per library, interleaved over rounds.   bash tools/attn_ab.sh <rounds> lib1.so lib2.so ...
set -u
rounds=$1; shift
export TMPDIR=/tmp
O=gpurun_out/attn_ab
mkdir -p $O
for r in $(seq 1 $rounds); do
  i=0
  for lib in "$@"; do
    i=$((i+1))
    d=$O/r${r}_v$i
    timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- \
      python tools/attn_time.py $lib > $d.log 2>&1 || exit 1
    f=$(find $d -name "*kernel_stats.csv" | head -1)
    echo "== round $r lib $i $lib" >> $O/summary.txt
    python tools/kstats.py "$f" 1 6 >> $O/summary.txt
  done
done
cat $O/summary.txt

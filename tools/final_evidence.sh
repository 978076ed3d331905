# Round-end evidence on one box: the C4 bench line (live roofline probe + CPU baseline), its rocprofv3
# kernel table and HBM PMC passes (tools/prof_round3.sh), then bench lines for the C4 trainer path and
# C2 / C3 / C5.                                bash tools/final_evidence.sh <round tag, e.g. r6>
set -u
R=${1:-r6}
export TMPDIR=/tmp
ROUND=$R bash tools/prof_round3.sh c4 || exit 1
O=gpurun_out/${R}_c4
timeout -k 10 300 python bench.py --config c4 --path trainer --no-cpu-baseline > $O/bench_trainer.json 2>> $O/bench.err || exit 1
for c in c2 c3 c5; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2>> $O/bench.err || exit 1
done
tail -c 600 $O/bench.json; for f in $O/bench_*.json; do python -c "import json,sys;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f',d['value'],d['ms_per_step'],d.get('roofline',{}).get('frac'))"; done

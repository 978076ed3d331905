"""Per-step kernel table from a rocprofv3 kernel_stats.csv.

    python tools/kstats.py <kernel_stats.csv> [steps] [rows] [--class prefix1,prefix2 ...]

`--class` sums every kernel whose name starts with one of the prefixes (the `rocprof_kernels`
of a bench line's roofline object), so the class's launches and ms per step can be read off the
same table the line cites.
"""
import csv
import sys

args = [a for a in sys.argv[1:]]
classes = []
while "--class" in args:
    i = args.index("--class")
    classes.append(tuple(args[i + 1].split(",")))
    del args[i:i + 2]
rows = list(csv.DictReader(open(args[0])))
steps = float(args[1]) if len(args) > 1 else 1
top = int(args[2]) if len(args) > 2 else 22
tot = sum(float(r['TotalDurationNs']) for r in rows)
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:top]:
    print(f"{float(r['TotalDurationNs'])/1e6/steps:8.3f} ms/step {float(r['Percentage']):6.2f}% "
          f"n={int(r['Calls'])/steps:6.1f}/step avg={float(r['AverageNs'])/1e3:8.1f}us  {r['Name'][:100]}")
print("total ms/step", tot / 1e6 / steps)
for pre in classes:
    sel = [r for r in rows if r['Name'].removeprefix('void ').startswith(pre)]
    ns = sum(float(r['TotalDurationNs']) for r in sel)
    n = sum(int(r['Calls']) for r in sel)
    print(f"class {'|'.join(p + '*' for p in pre)}: {n / steps:.1f} launches/step, {ns / 1e6 / steps:.3f} ms/step, "
          f"avg {ns / max(n, 1) / 1e3:.2f} us/launch")

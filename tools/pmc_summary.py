"""Average rocprofv3 --pmc counters per kernel name over the passes in a directory tree."""
import csv
import glob
import sys
from collections import defaultdict

root = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else ""
vals = defaultdict(lambda: defaultdict(list))
dur = defaultdict(list)
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        if filt not in name:
            continue
        vals[name[:90]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for f in glob.glob(f"{root}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if filt in r["Kernel_Name"]:
            dur[r["Kernel_Name"][:90]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for name, cs in vals.items():
    d = sorted(dur.get(name, [0]))
    print(f"== {name}  (median {d[len(d)//2]:.1f} us over {len(d)} launches)")
    for c, v in sorted(cs.items()):
        print(f"   {c:28s} {sum(v)/len(v):16.4g}")

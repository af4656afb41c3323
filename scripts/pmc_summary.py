"""Summarise rocprofv3 --pmc counter_collection.csv files per kernel (mean per dispatch)."""
import collections
import csv
import glob
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{root}/*/*_counter_collection.csv")):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        key = (r["Kernel_Name"].split("(")[0], r["Dispatch_Id"], r["Counter_Name"])
        per[key] += float(r["Counter_Value"])
    for (k, d, c), v in per.items():
        agg[k][c].append(v)
for k, cs in agg.items():
    print(k)
    for c, vs in sorted(cs.items()):
        print(f"   {c:28s} mean {sum(vs) / len(vs):14.4e}  n={len(vs)}")

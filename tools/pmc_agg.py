"""Aggregate rocprofv3 --pmc counter_collection CSVs per kernel (mean per dispatch)."""
import collections
import csv
import glob
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"].replace("(anonymous namespace)::", "")
        if n.startswith("void "):
            n = n[5:]
        n = n.split("(")[0].split("::")[-1]
        agg[n][r["Counter_Name"]].append(float(r["Counter_Value"]))
keys = sys.argv[2].split(",") if len(sys.argv) > 2 else sorted(agg)
for k in keys:
    d = agg.get(k)
    if d:
        print(k, {c: round(sum(v) / len(v)) for c, v in sorted(d.items())})

"""Summarise rocprofv3 --pmc CSVs: median per (kernel, counter) over dispatches."""
import csv
import glob
import statistics
import sys
from collections import defaultdict

root = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else ""
agg = defaultdict(list)
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if pat in r["Kernel_Name"]:
            name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
            agg[(name[-40:], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(agg.items()):
    print(f"{k:42s} {c:24s} n={len(v):4d} median={statistics.median(v):.6g} (first {v[0]:.6g})")

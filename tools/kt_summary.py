"""Per-kernel duration summary from a rocprofv3 kernel_trace.csv (median / mean / count)."""
import csv
import statistics
import sys
from collections import defaultdict

d = defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    d[r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")[-48:]].append(
        (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    print(f"{k:50s} n={len(v):5d} median={statistics.median(v):9.2f} us mean={sum(v)/len(v):9.2f} us "
          f"total={sum(v)/1e3:8.2f} ms")

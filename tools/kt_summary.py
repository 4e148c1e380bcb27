"""Per-kernel duration summary from a rocprofv3 kernel_trace.csv (median / mean / count).

`active` is the mean over launches longer than 20% of the median: round kernels launched past
convergence (the tail of the last batch) exit at their gate in a few microseconds and would
otherwise pull the plain mean below the duration of a real round.
"""
import csv
import statistics
import sys
from collections import defaultdict

d = defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    d[r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")[-48:]].append(
        (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    med = statistics.median(v)
    act = [x for x in v if x > 0.2 * med]
    print(f"{k:50s} n={len(v):5d} median={med:9.2f} us mean={sum(v)/len(v):9.2f} us "
          f"total={sum(v)/1e3:8.2f} ms active n={len(act)} mean={sum(act)/len(act):9.2f} us")

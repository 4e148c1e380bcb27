"""Turn rocprofv3 --pmc passes into profiles/<round>/pmc_summary.json and profiles/pmc_traffic.json
({workload: {kernel: HBM bytes per launch}}, read by bench.py for roofline.traffic).

FETCH_SIZE/WRITE_SIZE are in KB per dispatch.  On gfx950 FETCH_SIZE under-reports wide
coalesced reads by 2x (MI355X_MICROARCH.md §HBM); the factor actually applied is measured on
tools/microbench/membench's copy kernel (known 159 MB read) and stored as fetch_correction.

    python3 tools/make_pmc_traffic.py 'gpurun_out/c3pmc/pmc_*' profiles/round2/c3 "10000000 Imp3D push-sum" [calib glob]

PMC_STAT=active_mean: per (kernel, counter) the mean over the dispatches whose value is at least
1% of that counter's largest dispatch (the rounds that ran, not the gated-off launches past
convergence) instead of the median over all dispatches: for workloads whose rounds differ a lot
(C4 full gossip: 0.08 to 4.4 ms per round), so the figure matches the mean kernel time bench.py
divides by.
"""
import csv
import glob
import json
import os
import statistics
import sys
from collections import defaultdict

src, dst, workload = sys.argv[1], sys.argv[2], sys.argv[3]
calib = sys.argv[4] if len(sys.argv) > 4 else None


def medians(root, skip_first=1):
    """root: a directory or a glob of directories holding rocprofv3 counter_collection CSVs."""
    agg = defaultdict(list)
    files = [f for d in glob.glob(root) for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)]
    for f in files:
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
            agg[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
    if os.environ.get("PMC_STAT") == "active_mean":
        out = {}
        for (k, c), v in agg.items():
            top = max(v) if v else 0.0
            act = [x for x in v if x >= 0.01 * top] or v
            out[f"{k}|{c}"] = statistics.fmean(act)
        return out
    return {f"{k}|{c}": statistics.median(v[skip_first:] or v) for (k, c), v in agg.items()}


m = medians(src)
# PMC_FETCH_CORR: the FETCH_SIZE factor when no calibration run is given (2 for wide coalesced
# streaming reads, MI355X_MICROARCH.md; random narrow reads are uncalibrated: 1 = lower bound)
corr = float(os.environ.get("PMC_FETCH_CORR", "2.0"))
calib_info = None
if calib:
    cm = medians(calib, skip_first=0)
    fetch = [v for k, v in cm.items() if "copy_flat" in k and k.endswith("FETCH_SIZE")]
    if fetch:
        known = 9938376 * 16 / 1024.0  # KB read by copy_flat
        corr = known / fetch[0]
        calib_info = {"kernel": "membench copy_flat (16 B/lane coalesced read)", "fetch_kb": fetch[0],
                      "known_kb": known, "factor": corr}
out = {"workload": workload, "fetch_correction": corr, "calibration": calib_info,
       "statistic": os.environ.get("PMC_STAT", "median"), "medians": m}
os.makedirs(dst, exist_ok=True)
with open(os.path.join(dst, "pmc_summary.json"), "w") as f:
    json.dump(out, f, indent=1, sort_keys=True)
path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "pmc_traffic.json")
try:  # {workload: {kernel: entry}}: other workloads' entries are kept
    traffic = json.load(open(path))
    traffic = {w: e for w, e in traffic.items() if w != workload and isinstance(e, dict) and "workload" not in e}
except (OSError, ValueError):
    traffic = {}
cur = traffic.setdefault(workload, {})
for key, fetch in m.items():
    k, c = key.split("|")
    if c != "FETCH_SIZE":
        continue
    w = m.get(f"{k}|WRITE_SIZE")
    if w is None:
        continue
    short = k.split("::")[-1]
    cur[short] = {"fetch_kb": fetch, "write_kb": w, "fetch_correction": corr,
                  "hbm_bytes_per_launch": (fetch * corr + w) * 1024.0,
                  "source": os.path.join(dst, "pmc_summary.json")}
with open(path, "w") as f:
    json.dump(traffic, f, indent=1, sort_keys=True)
print(json.dumps(cur, indent=1))

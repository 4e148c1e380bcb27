"""Per-dispatch counter values of the kernels matching a pattern, in dispatch order.

    python3 tools/pmc_dispatch.py PMC_DIR [PMC_DIR ...] --kernel PATTERN [--min VALUE]

Each PMC_DIR holds one rocprofv3 --pmc pass (tools/gpu.sh pmc); the columns are the counters of
all the passes, joined on the dispatch's index among the matching kernels (every pass runs the
same program, so the i-th dispatch of a kernel is the same launch).  --min drops the rows whose
first counter is below VALUE (the early-exit launches of the gated passes).
"""
import argparse
import csv
import glob
from collections import defaultdict


def load(root, pat):
    rows = defaultdict(dict)
    for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if pat in r["Kernel_Name"]:
                key = (r["Kernel_Name"], int(r["Dispatch_Id"]))
                rows[key][r["Counter_Name"]] = rows[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    out = defaultdict(list)
    for (k, d), c in sorted(rows.items(), key=lambda x: x[0][1]):
        out[k].append(c)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--min", type=float, default=0.0)
    a = ap.parse_args()
    passes = [load(d, a.kernel) for d in a.dirs]
    for k in sorted(passes[0]):
        name = k.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
        n = min(len(p.get(k, [])) for p in passes)
        cols = [c for p in passes for c in sorted(p[k][0])]
        print(f"# {name}: {n} dispatches; " + " ".join(cols))
        for i in range(n):
            vals = [p[k][i][c] for p in passes for c in sorted(p[k][i])]
            if vals and vals[0] < a.min:
                continue
            print(f"{i:4d} " + " ".join(f"{v:14.6g}" for v in vals))


if __name__ == "__main__":
    main()

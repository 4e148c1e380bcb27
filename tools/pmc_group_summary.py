"""Whole-run HBM traffic of a GROUP of kernels that together make one round (e.g. full gossip's
k_gs_full4 plus the receipt tally's scans, placement and count passes, which run after it every
round, gated to a no-op in untallied rounds), from two rocprofv3 --pmc passes (FETCH_SIZE,
WRITE_SIZE; one run each) over the same run.

    python3 tools/pmc_group_summary.py FETCH_DIR WRITE_DIR OUT.json WORKLOAD NAME ROUNDS K1,K2,...

Every dispatch of K1..Kn in the run is summed (launches past convergence exit at their gate and add
a few KB), FETCH_SIZE doubled (gfx950 tallies 128 B read requests at 64 B: MI355X_MICROARCH.md
§HBM), and divided by ROUNDS, the run's round count.  Writes OUT.json (per-kernel totals and
dispatch counts) and the entry (WORKLOAD, NAME) of profiles/pmc_traffic.json, which bench.py reports
as roofline.traffic when the engine names its timed bracket NAME (gp_kstats.kernel).
"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FETCH_CORRECTION = 2.0


def totals(d, counter, kernels):
    out = {k: [0.0, 0] for k in kernels}
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
            name = name.replace("gp::", "")
            for k in kernels:
                if name == k or name.endswith("::" + k):
                    out[k][0] += float(r["Counter_Value"]) * 1024.0
                    out[k][1] += 1
    return out


def main():
    fdir, wdir, out, workload, group, rounds, klist = sys.argv[1:8]
    rounds = int(rounds)
    kernels = klist.split(",")
    fetch = totals(fdir, "FETCH_SIZE", kernels)
    write = totals(wdir, "WRITE_SIZE", kernels)
    per = {}
    for k in kernels:
        fb, fn = fetch[k]
        wb, wn = write[k]
        if fn == 0 or fn != wn:
            raise SystemExit(f"{k}: dispatch counts differ or are empty: FETCH {fn}, WRITE {wn}")
        per[k] = {"dispatches": fn, "fetch_bytes": FETCH_CORRECTION * fb, "write_bytes": wb,
                  "bytes_per_round": (FETCH_CORRECTION * fb + wb) / rounds}
    total = sum(v["bytes_per_round"] for v in per.values())
    summary = {"workload": workload, "group": group, "kernels": kernels, "rounds": rounds,
               "fetch_correction": FETCH_CORRECTION, "bytes_per_round": total, "per_kernel": per}
    os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
    with open(out, "w") as f:
        json.dump(summary, f, indent=1)
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            table = json.load(f)
    except (OSError, ValueError):
        table = {}
    entry = table.setdefault(workload, {}).setdefault(group, {})
    entry.clear()
    entry.update({"hbm_bytes_per_launch": total, "rounds": f"0..{rounds - 1} (whole run)",
                  "fetch_correction": FETCH_CORRECTION, "source": os.path.relpath(out, ROOT),
                  "kernels": {k: v["bytes_per_round"] for k, v in per.items()}})
    with open(path, "w") as f:
        json.dump(table, f, indent=1, sort_keys=True)
    print(f"{group}: {rounds} rounds, {total / 1e6:.1f} MB per round over the whole run")
    for k, v in per.items():
        print(f"  {k}: {v['dispatches']} dispatches, {v['bytes_per_round'] / 1e6:.1f} MB per round")


if __name__ == "__main__":
    main()

"""Durations of a kernel and the idle gaps between consecutive dispatches on its queue, from a
rocprofv3 --kernel-trace CSV: where a latency-bound run's time per round goes (the kernel itself or
the dispatch boundary).

    python3 tools/trace_gaps.py kt_kernel_trace.csv [NAME_SUBSTRING] [SKIP]
"""
import csv
import statistics
import sys


def main():
    path = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    skip = int(sys.argv[3]) if len(sys.argv) > 3 else 100
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[skip:]
    if not rows:
        raise SystemExit("no dispatches")
    sel = [r for r in rows if sub in r["Kernel_Name"]]
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in sel]
    gaps = [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3 for a, b in zip(rows, rows[1:])]
    span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e3
    print(f"{len(rows)} dispatches over {span:.1f} us; {len(sel)} matching {sub!r}")
    if dur:
        print(f"  duration us: median {statistics.median(dur):.2f} mean {statistics.fmean(dur):.2f}")
    print(f"  gap between consecutive dispatches us: median {statistics.median(gaps):.2f} "
          f"mean {statistics.fmean(gaps):.2f} (sum {sum(g for g in gaps if g > 0):.1f})")
    names = {}
    for r in rows:
        n = r["Kernel_Name"].split("(")[0].replace("void ", "")[-40:]
        names[n] = names.get(n, 0) + 1
    for n, c in sorted(names.items(), key=lambda x: -x[1])[:6]:
        print(f"  {c:7d} x {n}")


if __name__ == "__main__":
    main()

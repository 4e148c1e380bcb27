"""Per-round duration and HBM bytes of one round kernel over a whole run, side by side.

    python3 tools/round_series.py KT_TRACE_CSV PMC_RUN_JSON KERNEL [bucket] > table.txt

KT_TRACE_CSV: rocprofv3 --kernel-trace CSV of the run (tools/gpu.sh ktrun); PMC_RUN_JSON: the
per-round bytes of the same run (tools/pmc_run_summary.py, tools/gpu.sh pmcrun).  Dispatch order
is round order; buckets of `bucket` rounds (default 40) give mean us, MB and TB/s.
"""
import csv
import json
import sys


def main():
    trace, pmc, kernel = sys.argv[1:4]
    bucket = int(sys.argv[4]) if len(sys.argv) > 4 else 40
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(trace))
                  if kernel in r["Kernel_Name"])
    us = [(e - s) / 1e3 for s, e in rows]
    b = json.load(open(pmc))["per_round_bytes"]
    n = min(len(us), len(b))
    print(f"# {kernel}: {n} rounds; per bucket of {bucket}: mean duration, mean HBM bytes, rate")
    print(f"{'rounds':>11s} {'us':>8s} {'MB':>8s} {'TB/s':>6s}")
    for i in range(0, n, bucket):
        t = us[i:min(i + bucket, n)]
        x = b[i:min(i + bucket, n)]
        mt, mb = sum(t) / len(t), sum(x) / len(x)
        print(f"{i:5d}..{i + len(t) - 1:<5d} {mt:8.1f} {mb / 1e6:8.1f} {mb / (mt * 1e-6) / 1e12:6.2f}")
    print(f"# total {sum(us[:n]) / 1e3:.2f} ms; mean {sum(us[:n]) / n:.1f} us, "
          f"{sum(b[:n]) / n / 1e6:.1f} MB per round")


if __name__ == "__main__":
    main()

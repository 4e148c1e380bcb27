"""Per-round kernel time of a one-GPU run from a rocprofv3 kernel trace: the dispatches are assigned
to rounds by counting the round kernel's launches, and each round's time is split into the round
kernel and the passes after it.

    python3 tools/kt_round_series.py KT_CSV ROUND_KERNEL
"""
import csv
import sys


def name(r):
    return r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").replace("gp::", "")


def main():
    kt, rk = sys.argv[1:3]
    rows = sorted(csv.DictReader(open(kt)), key=lambda r: int(r["Start_Timestamp"]))
    rnd, per = -1, {}
    for r in rows:
        n = name(r)
        if n == rk:
            rnd += 1
        if rnd < 0:
            continue
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        per.setdefault(rnd, {}).setdefault(n, 0.0)
        per[rnd][n] += d
    total = 0.0
    print(f"# launch  {rk:>12s}  passes  total (us)")
    for k in sorted(per):
        s = sum(per[k].values())
        total += s
        print(f"{k:8d}  {per[k].get(rk, 0.0):12.1f}  {s - per[k].get(rk, 0.0):6.1f}  {s:8.1f}")
    print(f"# total {total / 1e3:.2f} ms over {len(per)} launches")


if __name__ == "__main__":
    main()

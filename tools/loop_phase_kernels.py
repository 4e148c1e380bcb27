"""Per-kernel cost of one rank-round by phase of a loopback shard run (tools/shard_loopback_prof.py
under rocprofv3 --kernel-trace): the dispatches are assigned to rounds by counting the round
kernel's launches (world per round, or world x pieces for a round in pieces, after the 8 warm-up
rounds), and each round to a phase by the global completion count before it (the run's trace from
--series).

    python3 tools/loop_phase_kernels.py KT_CSV SERIES_JSON ROUND_KERNEL [world] [warmup rounds, default 8] [bucket]

ROUND_KERNEL: one name, or several separated by commas (full gossip's ramp: k_gs_sparse_x,k_gs_full4x).
Warm-up rounds: the launches of run_local(max_rounds=8) per rank (gossip: 9, F(k) applies round k - 1).
PER_ROUND=N (environment): also every kernel of the first N rounds, round by round.

bucket: also the tail's rounds in buckets of that many (converged share, kernels and round kernel
per rank-round).
"""
import bisect
import csv
import json
import os
import statistics
import sys
from collections import defaultdict


def name(r):
    return r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").replace("gp::", "")


def main():
    kt, series, rks = sys.argv[1:4]
    rks = rks.split(",")
    world = int(sys.argv[4]) if len(sys.argv) > 4 else 8
    warm = int(sys.argv[5]) if len(sys.argv) > 5 else 8
    bucket = int(sys.argv[6]) if len(sys.argv) > 6 else 0
    d = json.load(open(series))
    trace, nodes = d["trace"], None
    rows = sorted(csv.DictReader(open(kt)), key=lambda r: int(r["Start_Timestamp"]))
    # launches of the round kernel per round: world x the round's pieces (8 warm-up rounds first)
    pieces = [d.get("warmup_pieces", 1)] * warm + d.get("pieces_per_round", [1] * len(d["trace"]))
    starts, acc = [], 0
    for k in pieces:
        starts.append(acc)
        acc += world * k
    seen, rnd = 0, -1
    per = defaultdict(lambda: defaultdict(float))  # round -> kernel -> us (all ranks)
    for r in rows:
        n = name(r)
        if any(n == rk or n.startswith(rk + "<") for rk in rks):  # (k_ps_quiet_x<false> / <true>)
            if seen < acc:
                rnd = bisect.bisect_right(starts, seen) - 1 - warm
            else:  # launched past the recorded rounds (one piece each)
                rnd = len(pieces) - warm + (seen - acc) // world
            seen += 1
        if rnd < 0:
            continue
        per[rnd][n] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    nodes = d.get("nodes") or max(trace)
    prev = [0] + trace[:-1]
    phases = {"dense (<1% converged)": lambda r, c: c * 100 < nodes,
              "mid (1-99% converged)": lambda r, c: nodes <= c * 100 < 99 * nodes,
              "tail (>=99% converged)": lambda r, c: c * 100 >= 99 * nodes,
              "rounds 0-18 (full gossip's ramp)": lambda r, c: r <= 18,
              "whole run": lambda r, c: True}
    for label, test in phases.items():
        rs = [r for r in per if r < len(prev) and test(r, prev[r])]
        if not rs:
            continue
        ks = sorted({k for r in rs for k in per[r]}, key=lambda k: -sum(per[r].get(k, 0.0) for r in rs))
        tot = statistics.fmean(sum(per[r].values()) for r in rs) / world
        print(f"{label}: {len(rs)} rounds, kernels per rank-round {tot:.1f} us, per rank over these rounds {tot * len(rs) / 1e3:.2f} ms")
        for k in ks:
            print(f"  {k:48s} {statistics.fmean(per[r].get(k, 0.0) for r in rs) / world:9.2f} us")
    per_round = int(os.environ.get("PER_ROUND", "0"))
    if per_round:  # the first rounds one by one: every kernel's time per rank-round (us)
        ks = sorted({k for r in per if r < per_round for k in per[r]})
        print("round " + " ".join(f"{k[:16]:>16s}" for k in ks))
        for r in sorted(x for x in per if x < per_round):
            print(f"{r:5d} " + " ".join(f"{per[r].get(k, 0.0) / world:16.2f}" for k in ks))
    if bucket:
        tail = sorted(r for r in per if r < len(prev) and prev[r] * 100 >= 99 * nodes)
        print(f"tail by {bucket} rounds: rounds, not converged before, kernels / round kernel per rank-round (us)")
        for i in range(0, len(tail), bucket):
            rs = tail[i:i + bucket]
            rkt = statistics.fmean(sum(v for k, v in per[r].items() if any(k == rk or k.startswith(rk + "<") for rk in rks))
                                   for r in rs)
            tot = statistics.fmean(sum(per[r].values()) for r in rs)
            print(f"  {rs[0]:5d}..{rs[-1]:<5d} {1 - prev[rs[0]] / nodes:8.5f} {tot / world:8.1f} {rkt / world:8.1f}")


if __name__ == "__main__":
    main()

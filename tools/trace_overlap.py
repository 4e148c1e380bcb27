"""Overlap of the exchange copies with the round kernels in a loopback kernel trace (rocprofv3
--kernel-trace CSV of tools/shard_loopback_prof.py): how much of the copies' time runs while a
kernel of the shards runs beside them (the copies of piece i beside the kernels of piece i+1,
DESIGN.md §6.11), and the busy time of each kind.

    python3 tools/trace_overlap.py kt_kernel_trace.csv
"""
import csv
import sys


def intervals(rows, pred):
    return sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows if pred(r["Kernel_Name"]))


def union(iv):
    out = []
    for s, e in iv:
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def covered(a, b):
    """Total length of a's intervals covered by the union b (both sorted; b disjoint)."""
    tot, j = 0, 0
    for s, e in a:
        while j < len(b) and b[j][1] <= s:
            j += 1
        k = j
        while k < len(b) and b[k][0] < e:
            tot += max(0, min(e, b[k][1]) - max(s, b[k][0]))
            k += 1
    return tot


rows = list(csv.DictReader(open(sys.argv[1])))
is_copy = lambda n: "copyBuffer" in n
setup = ("k_dst_", "k_scan_", "k_lpos", "k_link_hist", "k_sort_", "k_slot_owner", "k_add_u32", "k_load", "fillBuffer")
copies = intervals(rows, is_copy)
kern = intervals(rows, lambda n: not is_copy(n) and not any(s in n for s in setup))
ku = union(kern)
cu = union(copies)
ct = sum(e - s for s, e in cu)
kt = sum(e - s for s, e in ku)
ov = covered([tuple(x) for x in cu], ku)
print(f"copies: {len(copies)} dispatches, busy {ct / 1e6:.2f} ms; round kernels: busy {kt / 1e6:.2f} ms")
print(f"copy time beside a running kernel: {ov / 1e6:.2f} ms = {100.0 * ov / ct if ct else 0:.1f}% of the copies' busy time")

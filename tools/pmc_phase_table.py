"""Per-kernel hardware counters of a run, by phase of the run (rocprofv3 --pmc, one run per pass):
which bound a kernel of the round sits on in each phase.

    python3 tools/pmc_phase_table.py SERIES_JSON ROUND_KERNEL WORLD WARMUP KERNELS OUT.md PASS_DIR...

SERIES_JSON: the run's per-round completion counts ("trace"; tools/shard_loopback_prof.py --series
or tools/prof_run.py --series).  The dispatches of every pass are ordered by dispatch id and
assigned to rounds by counting ROUND_KERNEL's launches (WORLD per round, after WARMUP rounds), and
each round to a phase by the completion count before it, as tools/loop_phase_kernels.py does.
KERNELS: comma list of the kernels to tabulate.  Counters are summed per (phase, kernel) and
divided by the phase's rank-rounds; FETCH_SIZE is doubled (gfx950 tallies 128 B reads at 64 B,
MI355X_MICROARCH.md §HBM).  With WORLD = 1 and ROUND_KERNEL k_gs_full4 the one-GPU rounds are also
split into tallied rounds and atomic rounds (the tally placement pass runs over 3x its shortest
dispatch: tallied).
"""
import csv
import glob
import json
import statistics
import sys
from collections import defaultdict


def name(k):
    return k.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").replace("gp::", "")


def load(d):
    """dispatch id -> (kernel, {counter: value}) of one pass."""
    out = {}
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            did = int(r["Dispatch_Id"])
            k, c = out.setdefault(did, (name(r["Kernel_Name"]), {}))
            c[r["Counter_Name"]] = c.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return out


def rounds_of(disp, rk, world, warmup):
    """dispatch id -> round (None before the first real round)."""
    seen, rnd, out = 0, -1, {}
    rks = rk.split(",")  # (full gossip shards: the ramp's, the receipt wave's and the dense round kernels)
    for did in sorted(disp):
        k = disp[did][0]
        if any(k == x or k.startswith(x + "<") for x in rks):  # (k_ps_quiet_x<false> / <true>)
            rnd = seen // world - warmup
            seen += 1
        out[did] = rnd if rnd >= 0 else None
    return out


def main():
    series, rk, world, warmup, klist, out = sys.argv[1:7]
    dirs = sys.argv[7:]
    world, warmup = int(world), int(warmup)
    kernels = klist.split(",")
    d = json.load(open(series))
    trace = d["trace"]
    nodes = d.get("nodes") or max(trace)
    prev = [0] + trace[:-1]
    phases = {"dense (<1% converged)": lambda c: c * 100 < nodes,
              "mid (1-99% converged)": lambda c: nodes <= c * 100 < 99 * nodes,
              "tail (>=99% converged)": lambda c: c * 100 >= 99 * nodes,
              "whole run": lambda c: True}
    passes = [load(x) for x in dirs]
    # the one-GPU full gossip split: tallied / atomic rounds, by the tally placement pass, which
    # exits at once in a round that does not tally (tallied: over 3x its shortest dispatch)
    kind = {}
    if world == 1 and rk == "k_gs_full4":
        for p in passes:
            rr = rounds_of(p, rk, world, warmup)
            du = {rr[i]: c["GRBM_GUI_ACTIVE"] for i, (k, c) in p.items()
                  if k == "k_gs_tally_scatter_lds" and rr[i] is not None and "GRBM_GUI_ACTIVE" in c}
            if du:
                lo = min(du.values())
                kind = {r: "atomic" for r in set(rr.values()) if r is not None}
                kind.update({r: ("tallied" if v > 3 * lo else "atomic") for r, v in du.items()})
                break
        for label in ("tallied", "atomic"):
            phases[f"{label} rounds"] = (lambda lab: (lambda c, r=None: kind.get(r) == lab))(label)
    # (phase, kernel) -> counter -> [sum over each pass that holds it]: a counter collected in
    # several passes (GRBM_GUI_ACTIVE, SQ_WAVES) is averaged over them
    acc = defaultdict(lambda: defaultdict(list))
    nr = {}
    for p in passes:
        rr = rounds_of(p, rk, world, warmup)
        one = defaultdict(lambda: defaultdict(float))
        for label, test in phases.items():
            if label.endswith("rounds") and kind:
                rs = {r for r in set(rr.values()) if r is not None and r < len(prev) and test(0, r)}
            else:
                rs = {r for r in set(rr.values()) if r is not None and r < len(prev) and test(prev[r])}
            nr[label] = len(rs)
            for did, (k, c) in p.items():
                if k in kernels and rr[did] in rs:
                    for cn, v in c.items():
                        one[(label, k)][cn] += v
        for key, c in one.items():
            for cn, v in c.items():
                acc[key][cn].append(v)
    lines = [f"# Counters per rank-round by phase: {d.get('workload', '')} / {world}",
             "", f"({len(dirs)} rocprofv3 --pmc passes, one run each; {', '.join(dirs)})", ""]
    derived = [
        ("us (GRBM_GUI_ACTIVE / 8 XCD / 2.4 GHz)", lambda c: c.get("GRBM_GUI_ACTIVE", 0) / 8 / 2400.0 if "GRBM_GUI_ACTIVE" in c else None),
        ("waves", lambda c: c.get("SQ_WAVES")),
        ("VMEM rd insts / wave", lambda c: c["SQ_INSTS_VMEM_RD"] / c["SQ_WAVES"] if "SQ_INSTS_VMEM_RD" in c and c.get("SQ_WAVES") else None),
        ("VMEM wr insts / wave", lambda c: c["SQ_INSTS_VMEM_WR"] / c["SQ_WAVES"] if "SQ_INSTS_VMEM_WR" in c and c.get("SQ_WAVES") else None),
        ("VALU insts / wave", lambda c: c["SQ_INSTS_VALU"] / c["SQ_WAVES"] if "SQ_INSTS_VALU" in c and c.get("SQ_WAVES") else None),
        ("LDS insts / wave", lambda c: c["SQ_INSTS_LDS"] / c["SQ_WAVES"] if "SQ_INSTS_LDS" in c and c.get("SQ_WAVES") else None),
        ("LDS bank-conflict cycles / LDS-array cycles", lambda c: c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"] if c.get("SQ_LDS_IDX_ACTIVE") else None),
        ("wave time parked (SQ_WAIT_ANY / SQ_WAVE_CYCLES)", lambda c: c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"] if c.get("SQ_WAVE_CYCLES") and "SQ_WAIT_ANY" in c else None),
        ("wave time issue-stalled (SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES)", lambda c: c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"] if c.get("SQ_WAVE_CYCLES") and "SQ_WAIT_INST_ANY" in c else None),
        ("wave time issuing (SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES)", lambda c: c["SQ_ACTIVE_INST_ANY"] / c["SQ_WAVE_CYCLES"] if c.get("SQ_WAVE_CYCLES") and "SQ_ACTIVE_INST_ANY" in c else None),
        ("TA busy (TA_TA_BUSY_sum / GRBM_GUI_ACTIVE / 256 CU)", lambda c: c["TA_TA_BUSY_sum"] / c["GRBM_GUI_ACTIVE"] / 32.0 if c.get("GRBM_GUI_ACTIVE") and "TA_TA_BUSY_sum" in c else None),
        ("TD busy (TD_TD_BUSY_sum / GRBM_GUI_ACTIVE / 256 CU)", lambda c: c["TD_TD_BUSY_sum"] / c["GRBM_GUI_ACTIVE"] / 32.0 if c.get("GRBM_GUI_ACTIVE") and "TD_TD_BUSY_sum" in c else None),
        ("atomics at memory (TCC_EA0_ATOMIC_sum)", lambda c: c.get("TCC_EA0_ATOMIC_sum")),
        ("atomics in L2 (TCC_ATOMIC_sum)", lambda c: c.get("TCC_ATOMIC_sum")),
        ("L2 hit rate", lambda c: c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"]) if c.get("TCC_HIT_sum", 0) + c.get("TCC_MISS_sum", 0) else None),
        ("HBM read MB (2 x FETCH_SIZE)", lambda c: 2.0 * c["FETCH_SIZE"] / 1024.0 if "FETCH_SIZE" in c else None),
        ("HBM write MB (WRITE_SIZE)", lambda c: c["WRITE_SIZE"] / 1024.0 if "WRITE_SIZE" in c else None),
    ]
    ratio_rows = {r[0] for r in derived if r[0].startswith(("VMEM", "VALU", "LDS", "wave time", "TA busy", "TD busy", "L2 hit"))}
    js = {}
    for label in phases:
        n = nr.get(label, 0)
        if not n:
            continue
        ks = [k for k in kernels if (label, k) in acc]
        if not ks:
            continue
        lines += [f"## {label}: {n} rounds", "", "| per rank-round | " + " | ".join(ks) + " |",
                  "|---|" + "---|" * len(ks)]
        for row, f in derived:
            vals = []
            for k in ks:
                c = {cn: statistics.fmean(v) for cn, v in acc[(label, k)].items()}
                scale = 1.0 if row in ratio_rows else 1.0 / (n * world)
                try:
                    v = f(c)
                except (KeyError, ZeroDivisionError):
                    v = None
                vals.append(None if v is None else v * scale)
            if all(v is None for v in vals):
                continue
            js.setdefault(label, {})[row] = dict(zip(ks, vals))
            lines.append(f"| {row} | " + " | ".join("—" if v is None else (f"{v:.3f}" if abs(v) < 10 else f"{v:,.0f}") for v in vals) + " |")
        lines.append("")
    open(out, "w").write("\n".join(lines) + "\n")
    json.dump(js, open(out.rsplit(".", 1)[0] + ".json", "w"), indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main()

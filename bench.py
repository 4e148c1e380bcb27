"""bench.py — BASELINE.json's headline: node-updates/s and wall time to push-sum convergence,
imperfect-3D, 10M nodes (configs[2]: `10000000 Imp3D push-sum`, 9,938,375 nodes, G = 239).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload auto|c3|c4|c5|custom]
                    [--n N --topology T --algorithm A --window R] [--no-cpu-baseline]

Workloads:
  c3    `10000000 Imp3D push-sum` to convergence — the headline, the N = 1 default.  One step
        = one complete simulation from the reference's initial state (S_i = i, W_i = 1,
        termRound = 1; program.fs:78-79,107-108): reset + run.  The topology (extra links,
        link CSR) is built once before timing, as the reference starts its timer after
        building the actors (program.fs:317).
  c5    `1000000000 Imp3D push-sum` over a fixed window of --window rounds (default 50): the
        north star's 1B-node graph — the N > 1 default (strong scaling: the same graph split
        over N ranks), and runnable at N = 1 for the one-GPU point of that curve.
  c4    `100000000 full gossip` to convergence (19 B per node-update roofline, int atomics).
  custom  --n / --topology / --algorithm [/ --window].

N = 1: the single-GPU engine (gp_step).  N > 1 (launched by torch.distributed.run, one rank per
GPU): node-range shards (whole z-planes), one fixed-size RCCL all-to-all per round (DESIGN.md
§6); value = global actors x rounds / max-over-ranks wall time, and `per_rank` reports rank 0's
round time split into round kernels / all-to-all / unpack plus the bytes it exchanges per round.
Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "cop5615-gossip_protocol_amd"))

METRIC = "node-updates/sec + wall-time to push-sum convergence, imperfect3D 10M nodes"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
CPU_BASELINE_MAX_N = 200_000_000

WORKLOADS = {  # name: (n_arg, topology, algorithm, window rounds or None = to convergence)
    "c3": (10_000_000, "Imp3D", "push-sum", None),
    "c5": (1_000_000_000, "Imp3D", "push-sum", 50),
    "c4": (100_000_000, "full", "gossip", None),
}


def survey_bytes_per_update(topology, algorithm):
    """algorithmic HBM bytes per node-update (the roofline's unit)."""
    if algorithm == "gossip":
        return 19.0
    return 112.0 if topology == "Imp3D" else 108.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", choices=["auto", "c3", "c4", "c5", "custom"], default="auto",
                    help="auto: c3 on one GPU, c5 (strong scaling) on several")
    ap.add_argument("--n", type=int, default=10_000_000, help="custom: numNodes (argv[1]) of the whole graph")
    ap.add_argument("--topology", default="Imp3D")
    ap.add_argument("--algorithm", default="push-sum")
    ap.add_argument("--window", type=int, default=None, help="fixed round window (default: to convergence; c5: 50)")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="CPU baseline sample budget")
    ap.add_argument("--no-kernel-timing", action="store_true")
    ap.add_argument("--engine", choices=["auto", "shard"], default="auto",
                    help="auto: single-GPU engine at N=1, shards at N>1; shard: shards also at N=1")
    return ap.parse_args()


def workload(args, world):
    name = args.workload
    if name == "auto":
        name = "c3" if world == 1 else "c5"
    if name == "custom":
        return name, args.n, args.topology, args.algorithm, args.window
    n, topo, algo, window = WORKLOADS[name]
    return name, n, topo, algo, args.window if args.window is not None else window


def pmc_traffic(kernels, wl: str):
    """HBM bytes per round of `kernels` (summed) from the committed rocprofv3 PMC summary
    (profiles/pmc_traffic.json {workload: {kernel: ...}}, made by tools/make_pmc_traffic.py), or
    None when the workload or a kernel has no entry."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    per = d.get(wl)
    if not isinstance(per, dict):
        return None
    total = 0.0
    for k in kernels:
        e = per.get(k)
        if not e:
            return None
        total += e["hbm_bytes_per_launch"]
    return total


def cpu_baseline(n, topology, algorithm, seed, budget_s, window):
    """The CPU oracle (OpenMP pull mode, same seeds) on a bounded sample of the same workload:
    the first R rounds, R chosen so the sample takes about budget_s seconds."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # test infrastructure: timed here as the CPU baseline only

    threads = int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1)
    threads = max(1, min(threads, os.cpu_count() or 1))
    sim = oracle.OracleSim(n, topology, algorithm, seed=seed)
    sim.step(1, threads=threads)  # builds the in-neighbour CSR outside the timed sample
    t0 = time.perf_counter()
    rounds = 0
    chunk = 2
    cap = (window - 1) if window else 2000
    while True:
        sim.step(min(chunk, cap - rounds), threads=threads)
        rounds = int(sim.status.round) - 1
        el = time.perf_counter() - t0
        if el >= budget_s or sim.status.converged or rounds >= cap:
            break
        chunk = max(1, min(64, int(chunk * max(1.5, min(4.0, budget_s / max(el, 1e-3) * 0.5)))))
    el = time.perf_counter() - t0
    value = sim.actors * rounds / el
    sim.close()
    return {"value": value, "unit": "node-updates/s", "cores": threads, "kind": "port",
            "sample": f"rounds 1..{rounds} of `{n} {topology} {algorithm}` seed {seed} "
                      f"({sim.actors} actors), oracle/gp_oracle.c OpenMP pull mode, {el:.1f} s"}


def roofline(ks, bytes_per_update, actors, wl):
    """Round roofline: SURVEY §8(d) bytes per node-update x this rank's actors over the
    measured duration of one round = the round kernel + the pass that completes it (link
    scatter), both timed with hipEvents on the engine's stream inside the timed steps."""
    if not ks["launches"]:
        return None
    round_ms = ks["avg_ms"] + ks["aux_avg_ms"]
    algo_bytes = bytes_per_update * actors
    achieved = algo_bytes / (round_ms * 1e-3) / 1e9
    kernels = [ks["kernel"]] + ([ks["aux_kernel"]] if ks["aux_kernel"] else [])
    traffic = pmc_traffic(kernels, wl)
    return {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
            "kernel": " + ".join(kernels), "avg_kernel_ms": round(ks["avg_ms"], 5),
            "avg_aux_ms": round(ks["aux_avg_ms"], 5), "round_ms": round(round_ms, 5),
            "bytes_per_launch": algo_bytes, "bytes_per_update": bytes_per_update, "launches": ks["launches"],
            "layout_bytes_per_launch": ks["bytes_per_launch"],
            "layout_frac": round(ks["bytes_per_launch"] / (ks["avg_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}


def strong_scaling_base(name):
    """The one-GPU point of the strong-scaling curve of workload `name` (N > 1 runs split one
    graph): the committed N = 1 bench line of the same workload, so a reader can form the
    efficiency against the same graph (the driver's N = 1 run is the c3 headline)."""
    path = os.path.join(ROOT, "profiles", "round2", name, "bench_line_n1.json")
    try:
        with open(path) as f:
            d = json.load(f)
        return {"value": d["value"], "unit": d["unit"], "workload": d["config"]["workload"],
                "source": os.path.relpath(path, ROOT)}
    except (OSError, ValueError, KeyError):
        return None


def progress(rank, msg, t0=time.perf_counter()):
    """Rank 0 stage marks on stderr (stdout carries only the JSON line)."""
    if rank == 0:
        print(f"[bench {time.perf_counter() - t0:7.1f} s] {msg}", file=sys.stderr, flush=True)


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    use_shards = world > 1 or args.engine == "shard"
    if use_shards:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        progress(rank, f"process group up (nccl, world {world})")
    else:
        torch.cuda.set_device(0)
    from gossip_amd import Simulator, sharded

    name, n_arg, topology, algorithm, window = workload(args, world)
    progress(rank, f"{name}: {n_arg} {topology} {algorithm} on {world} GPU(s)")
    cap = window if window else 1 << 40
    timing = not args.no_kernel_timing
    timer = None
    if use_shards:
        eng = sharded.HipShard(n_arg, topology, algorithm, rank=rank, world=world, seed=args.seed,
                               device=local, kernel_timing=timing)
        transport = sharded.TorchTransport()
        own = eng.hi - eng.lo

        def one_step(t=None):
            eng.reset()
            st = sharded.run(eng, transport, max_rounds=cap, timer=t)
            return int(st.round), bool(st.converged)
    else:
        stream = torch.cuda.Stream()
        eng = Simulator(n_arg, topology, algorithm, seed=args.seed, device=local,
                        kernel_timing=timing, stream=stream.cuda_stream)
        own = eng.actors

        def one_step(t=None):
            eng.reset()
            st = eng.step(cap)
            return int(st.round), bool(st.converged)

    progress(rank, f"engine ready ({eng.actors} actors, {own} on this rank)")
    for _ in range(args.warmup):
        one_step()
    eng.kernel_stats(reset=True)
    progress(rank, f"{args.warmup} warmup step(s) done")

    def barrier():
        if use_shards:
            dist.barrier()
        torch.cuda.synchronize()

    rounds_total = 0
    converged = True
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        r, c = one_step()
        rounds_total += r
        converged &= c
    barrier()
    elapsed = time.perf_counter() - t0
    progress(rank, f"{args.steps} timed step(s): {elapsed * 1e3:.1f} ms")
    updates = float(eng.actors) * rounds_total  # global actors: every rank agrees on the rounds
    if use_shards:
        t = torch.tensor([elapsed], device="cuda", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ks = eng.kernel_stats()
    per_rank = None
    if use_shards:  # one extra, untimed step with sampled per-phase events (rank 0 reports)
        timer = sharded.PhaseTimer()
        one_step(timer)
        per_rank = dict(timer.means(), actors=own, bytes_sent_per_round=sum(eng.send_splits),
                        bytes_received_per_round=sum(eng.recv_splits), world=world)
    wl = f"{n_arg} {topology} {algorithm}"
    out = None
    if rank == 0:
        roof = roofline(ks, survey_bytes_per_update(topology, algorithm), own, wl)
        cpu = None
        # the oracle holds the whole graph in host memory and builds it serially: beyond ~2e8
        # nodes its setup alone outlasts a bounded sample, so C5 (1e9) reports none
        if world == 1 and not args.no_cpu_baseline and n_arg <= CPU_BASELINE_MAX_N:
            progress(rank, "CPU baseline sample")
            cpu = cpu_baseline(n_arg, topology, algorithm, args.seed, args.cpu_seconds, window)
        rounds_per_step = rounds_total / max(1, args.steps)
        scaling = "weak" if world == 1 else "strong"
        out = {
            "metric": METRIC,
            "value": updates / elapsed,
            "unit": "node-updates/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (reference initial state S_i=i, W_i=1; Philox seed %d)" % args.seed,
            "config": {"workload": wl + (f", {window}-round window" if window else ", to convergence"),
                       "name": name, "actors": eng.actors, "nodes": eng.nodes,
                       "actors_per_gpu": own, "grid": int(eng.layout.grid),
                       "rounds_per_step": rounds_per_step, "converged": converged,
                       "parallelism": f"node-range shards x{world}, RCCL all-to-all" if use_shards else "single"},
            "wall_time_to_convergence_ms": elapsed * 1e3 / args.steps if not window else None,
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        if per_rank:
            out["per_rank"] = per_rank
        if world > 1:
            out["strong_scaling_base"] = strong_scaling_base(name)
        print(json.dumps(out), flush=True)
    eng.close()
    if use_shards:
        dist.destroy_process_group()
    return out


if __name__ == "__main__":
    main()

"""bench.py — BASELINE.json's headline: node-updates/s and wall time to push-sum convergence,
imperfect-3D, 10M nodes (configs[2]: `10000000 Imp3D push-sum`, 9,938,375 nodes, G = 239).

One step = one complete simulation to convergence from the reference's initial state
(S_i = i, W_i = 1, termRound = 1; program.fs:78-79,107-108): reset + run.  Topology build
(extra links, link CSR) happens once before timing, as the reference starts its timer after
building the actors (program.fs:317).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--n 10000000] [--no-cpu-baseline]

N = 1: the single-GPU engine (gp_step).  N > 1 (launched by torch.distributed.run, one rank per
GPU): ONE graph of N x 10M nodes (weak scaling) split into node-range shards (whole z-planes),
one fixed-size RCCL all-to-all per round.  value = global actors x rounds /
max-over-ranks wall time.  Rank 0 prints ONE JSON line.
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
    ap.add_argument("--n", type=int, default=10_000_000, help="numNodes per GPU (argv[1])")
    ap.add_argument("--topology", default="Imp3D")
    ap.add_argument("--algorithm", default="push-sum")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="CPU baseline sample budget")
    ap.add_argument("--no-kernel-timing", action="store_true")
    ap.add_argument("--engine", choices=["auto", "shard"], default="auto",
                    help="auto: single-GPU engine at N=1, shards at N>1; shard: shards also at N=1")
    return ap.parse_args()


def pmc_traffic(kernels, workload: str):
    """HBM bytes per round of `kernels` (summed) from the committed rocprofv3 PMC summary
    (profiles/pmc_traffic.json, made by tools/make_pmc_traffic.py), or None."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    total = 0.0
    for k in kernels:
        e = d.get(k)
        if not e or e.get("workload") != workload:
            return None
        total += e["hbm_bytes_per_launch"]
    return total


def cpu_baseline(n, topology, algorithm, seed, budget_s):
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
    while True:
        sim.step(chunk, threads=threads)
        rounds += chunk
        el = time.perf_counter() - t0
        if el >= budget_s or sim.status.converged or rounds >= 2000:
            break
        chunk = max(1, min(64, int(chunk * max(1.5, min(4.0, budget_s / max(el, 1e-3) * 0.5)))))
    el = time.perf_counter() - t0
    value = sim.actors * rounds / el
    sim.close()
    return {"value": value, "unit": "node-updates/s", "cores": threads, "kind": "port",
            "sample": f"rounds 1..{rounds} of `{n} {topology} {algorithm}` seed {seed} "
                      f"({sim.actors} actors), oracle/gp_oracle.c OpenMP pull mode, {el:.1f} s"}


def roofline(ks, bytes_per_update, actors, workload):
    """Round roofline: SURVEY §8(d) bytes per node-update x this rank's actors over the
    measured duration of one round = the round kernel + the pass that completes it (link
    scatter), both timed with hipEvents on the engine's stream inside the timed steps."""
    if not ks["launches"]:
        return None
    round_ms = ks["avg_ms"] + ks["aux_avg_ms"]
    algo_bytes = bytes_per_update * actors
    achieved = algo_bytes / (round_ms * 1e-3) / 1e9
    kernels = [ks["kernel"]] + ([ks["aux_kernel"]] if ks["aux_kernel"] else [])
    traffic = pmc_traffic(kernels, workload)
    return {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
            "kernel": " + ".join(kernels), "avg_kernel_ms": round(ks["avg_ms"], 5),
            "avg_aux_ms": round(ks["aux_avg_ms"], 5), "round_ms": round(round_ms, 5),
            "bytes_per_launch": algo_bytes, "bytes_per_update": bytes_per_update, "launches": ks["launches"],
            "layout_bytes_per_launch": ks["bytes_per_launch"],
            "layout_frac": round(ks["bytes_per_launch"] / (ks["avg_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}


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
    else:
        torch.cuda.set_device(0)
    from gossip_amd import Simulator, sharded

    timing = not args.no_kernel_timing
    n_arg = args.n * world  # weak scaling: ~args.n nodes per GPU
    if use_shards:
        eng = sharded.HipShard(n_arg, args.topology, args.algorithm, rank=rank, world=world, seed=args.seed,
                               device=local, kernel_timing=timing)
        transport = sharded.TorchTransport()
        own = eng.hi - eng.lo

        def one_step():
            eng.reset()
            st = sharded.run(eng, transport)
            return int(st.round), bool(st.converged)
    else:
        stream = torch.cuda.Stream()
        eng = Simulator(n_arg, args.topology, args.algorithm, seed=args.seed, device=local,
                        kernel_timing=timing, stream=stream.cuda_stream)
        own = eng.actors

        def one_step():
            eng.reset()
            st = eng.step()
            return int(st.round), bool(st.converged)

    for _ in range(args.warmup):
        one_step()
    eng.kernel_stats(reset=True)

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
    updates = float(eng.actors) * rounds_total  # global actors: every rank agrees on the rounds
    if use_shards:
        t = torch.tensor([elapsed], device="cuda", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ks = eng.kernel_stats()
    workload = f"{n_arg} {args.topology} {args.algorithm}"
    out = None
    if rank == 0:
        roof = roofline(ks, survey_bytes_per_update(args.topology, args.algorithm), own, workload)
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(n_arg, args.topology, args.algorithm, args.seed, args.cpu_seconds)
        rounds_per_step = rounds_total / max(1, args.steps)
        out = {
            "metric": METRIC,
            "value": updates / elapsed,
            "unit": "node-updates/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (reference initial state S_i=i, W_i=1; Philox seed %d)" % args.seed,
            "config": {"workload": workload, "actors": eng.actors, "nodes": eng.nodes,
                       "actors_per_gpu": own, "grid": int(eng.layout.grid),
                       "rounds_to_convergence": rounds_per_step, "converged": converged,
                       "parallelism": f"node-range shards x{world}, RCCL all-to-all" if use_shards else "single"},
            "wall_time_to_convergence_ms": elapsed * 1e3 / args.steps,
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    eng.close()
    if use_shards:
        dist.destroy_process_group()
    return out


if __name__ == "__main__":
    main()

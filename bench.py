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

N = 1: the single-GPU engine (gp_step).  N > 1, two launch forms, both split ONE graph (c5 by
default: strong scaling) into node-range shards (whole z-planes) with one fixed-size exchange per
round:
  * `torch.distributed.run ... bench.py --gpus N` (the driver's form): one process per GPU, the
    exchange is torch's all_to_all_single over RCCL;
  * `python bench.py --gpus N` (no WORLD_SIZE): ONE process drives N GPUs through the library's
    own multi-GPU engine (gp_config.num_gpus = N: ncclCommInitAll + grouped ncclSend/ncclRecv,
    SURVEY.md §8b).  --one-device puts the N shards on device 0 with device copies in place of
    RCCL (the same code path on a one-GPU box).  Fewer than N devices is an error, never a silent
    one-GPU run.
Either way the job first times the same window on device 0 alone with the single-GPU engine
(`strong_scaling_base`, same job, before any shard exists), value = global actors x rounds /
max-over-ranks wall time, and `per_rank` reports rank 0's round time.  Rank 0 prints ONE JSON
line.
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


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="GPUs of this node: torch.distributed.run ranks, or (no WORLD_SIZE) one process "
                         "driving N devices through the library's multi-GPU engine (bit-exact with N shards "
                         "on one GPU; an RCCL exchange between physical GPUs is untested so far)")
    ap.add_argument("--one-device", action="store_true",
                    help="--gpus N without torch.distributed: the N shards on device 0, exchange by "
                         "device copies (tests the multi-GPU engine on a one-GPU box)")
    ap.add_argument("--no-base", action="store_true", help="N > 1: skip the same-job one-GPU base")
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
    return ap.parse_args(argv)


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
    (profiles/pmc_traffic.json {workload: {kernel: ...}}, made by tools/pmc_run_summary.py over a
    whole run, or tools/make_pmc_traffic.py), and the rounds that figure covers; (None, None) when
    the workload or a kernel has no entry."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None, None
    per = d.get(wl)
    if not isinstance(per, dict):
        return None, None
    total, spans = 0.0, []
    for k in kernels:
        e = per.get(k)
        if not e:
            return None, None
        total += e["hbm_bytes_per_launch"]
        span = e.get("rounds", "median of the first 60 rounds")
        spans.append(f"{span}, {e['source']}" if e.get("source") else span)
    return total, "; ".join(sorted(set(spans)))


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
    return {"value": value, "unit": "node-updates/s", "cores": threads, "kind": "port", "rounds": rounds,
            "sample": f"rounds 1..{rounds} of `{n} {topology} {algorithm}` seed {seed} "
                      f"({sim.actors} actors), oracle/gp_oracle.c OpenMP pull mode, {el:.1f} s"}


def gpu_same_window(eng, rounds, reps=3):
    """The GPU engine over the CPU sample's window (rounds 1..R of the same run, R from
    cpu_baseline): the same-span rate a GPU/CPU ratio should use (the whole-run `value` includes
    the cheap converged tail, which the CPU sample never reaches)."""
    import torch

    best = None
    for _ in range(reps):
        eng.reset()
        eng.step(1)  # round 0, untimed as on the CPU side
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        st = eng.step(rounds)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        assert int(st.round) - 1 == rounds, (st.round, rounds)
        best = el if best is None else min(best, el)
    return eng.actors * rounds / best


def roofline(ks, bytes_per_update, actors, wl, rounds=None):
    """Round roofline: SURVEY §8(d) bytes per node-update x the node-updates one launch performs
    over the measured duration of one round = the round kernel + the pass that completes it (link
    scatter), both timed with hipEvents on the engine's stream inside the timed steps.  The
    node-updates per launch are the engine's own count (gp_kstats.work_per_launch): every actor of
    the range, except that the one-GPU quiet-tail kernel counts the actors it walks, so the
    converged tail, where a round touches a few percent of the actors, is not credited 112 B for
    every actor (that figure, `frac_all_actors`, exceeds 1 once the tail is cheap)."""
    if not ks["launches"]:
        return None
    round_ms = ks["avg_ms"] + ks["aux_avg_ms"]
    units = ks.get("work_per_launch") or float(actors)
    algo_bytes = bytes_per_update * units
    achieved = algo_bytes / (round_ms * 1e-3) / 1e9
    kernels = [ks["kernel"]] + ([ks["aux_kernel"]] if ks["aux_kernel"] else [])
    traffic, traffic_rounds = pmc_traffic(kernels, wl)
    # measured HBM bytes (PMC) over their rounds' mean time: the fraction of peak the kernel moves
    measured = traffic / (round_ms * 1e-3) / 1e9 / HBM_PEAK_GBS if traffic else None
    return {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_rounds": traffic_rounds,
            "hbm_measured_frac": round(measured, 4) if measured else None,
            "kernel": " + ".join(kernels), "avg_kernel_ms": round(ks["avg_ms"], 5),
            "avg_aux_ms": round(ks["aux_avg_ms"], 5), "round_ms": round(round_ms, 5),
            "bytes_per_launch": algo_bytes, "bytes_per_update": bytes_per_update,
            "updates_per_launch": round(units, 1), "actors": actors, "launches": ks["launches"],
            # the launches the hipEvent brackets cover vs the rounds the timed steps ran: one GPU
            # times every round (64-round groups); a shard samples every 8th round
            "timed_launches": ks["launches"], "rounds": rounds,
            "frac_all_actors": round(bytes_per_update * actors / (round_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "layout_bytes_per_launch": ks["bytes_per_launch"],
            "layout_frac": round(ks["bytes_per_launch"] / (ks["avg_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}


def single_gpu_window(n_arg, topology, algorithm, seed, window, steps, warmup, device=0):
    """The one-GPU point of a strong-scaling curve, measured in the same job before any shard
    exists: the single-GPU engine (gp_step) on `device` over the same graph and window, then
    freed.  Returns value (node-updates/s), ms per step and rounds per step."""
    import torch

    from gossip_amd import Simulator

    cap = window if window else 1 << 40
    stream = torch.cuda.Stream(device)
    eng = Simulator(n_arg, topology, algorithm, seed=seed, device=device, stream=stream.cuda_stream)
    try:
        for _ in range(warmup):
            eng.reset()
            eng.step(cap)
        rounds = 0
        torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        for _ in range(steps):
            eng.reset()
            rounds += int(eng.step(cap).round)
        torch.cuda.synchronize(device)
        el = time.perf_counter() - t0
        return {"value": eng.actors * rounds / el, "unit": "node-updates/s", "ms_per_step": el * 1e3 / steps,
                "rounds_per_step": rounds / steps, "steps": steps,
                "workload": f"{n_arg} {topology} {algorithm}" + (f", {window}-round window" if window else ""),
                "engine": f"single-GPU gp_step on device {device}, same job, before the shards were built"}
    finally:
        eng.close()
        del eng
        torch.cuda.synchronize(device)
        torch.cuda.empty_cache()


def progress(rank, msg, t0=time.perf_counter()):
    """Rank 0 stage marks on stderr (stdout carries only the JSON line)."""
    if rank == 0:
        print(f"[bench {time.perf_counter() - t0:7.1f} s] {msg}", file=sys.stderr, flush=True)


def fail(msg):
    print(f"bench.py: {msg}", file=sys.stderr, flush=True)
    raise SystemExit(2)


def roofline_for(ks, topology, algorithm, actors, wl, rounds=None):
    return roofline(ks, survey_bytes_per_update(topology, algorithm), actors, wl, rounds)


def base_line(args, rank, n_arg, topology, algorithm, window, devices):
    """The same-job one-GPU point (rank 0 / device 0), or None (skipped, or more nodes than one
    GPU's 288 GB hold)."""
    if args.no_base or rank != 0:
        return None
    progress(rank, "one-GPU base: the same window on device 0 alone")
    b = single_gpu_window(n_arg, topology, algorithm, args.seed, window, args.steps, args.warmup, device=0)
    progress(rank, f"one-GPU base: {b['value']:.3e} node-updates/s, {b['ms_per_step']:.1f} ms per step")
    return b


def attach_base(out, base, value, n):
    if base:
        base = dict(base)
        base["t1_over_n_tn"] = value / (n * base["value"])  # = T1 / (N * TN): same rounds, same graph
        out["strong_scaling_base"] = base


def emit_line(args, *, name, n_arg, topology, algorithm, window, eng_actors, eng_nodes, grid, own, n_gpus, updates,
              elapsed, rounds_total, converged, parallelism, ks, cpu=None, extra=None):
    wl = f"{n_arg} {topology} {algorithm}"
    out = {
        "metric": METRIC,
        "value": updates / elapsed,
        "unit": "node-updates/s",
        "n_gpus": n_gpus,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": "weak" if n_gpus == 1 else "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (reference initial state S_i=i, W_i=1; Philox seed %d)" % args.seed,
        "config": {"workload": wl + (f", {window}-round window" if window else ", to convergence"),
                   "name": name, "actors": eng_actors, "nodes": eng_nodes,
                   "actors_per_gpu": own, "grid": grid,
                   "rounds_per_step": rounds_total / max(1, args.steps), "converged": converged,
                   "parallelism": parallelism},
        "wall_time_to_convergence_ms": elapsed * 1e3 / args.steps if not window else None,
        "roofline": roofline_for(ks, topology, algorithm, own, wl, rounds_total),
        "cpu_baseline": cpu,
    }
    if extra:
        out.update(extra)
    return out


def main_group(args):
    """--gpus N in ONE process: the library's multi-GPU engine (gp_config.num_gpus = N)."""
    import torch

    from gossip_amd import Simulator, sharded

    N = args.gpus
    ndev = torch.cuda.device_count()
    if args.one_device:
        if ndev < 1:
            fail(f"--gpus {N} --one-device needs one GPU; {ndev} visible")
    elif ndev < N:
        fail(f"--gpus {N} needs {N} GPUs in this process; {ndev} visible "
             f"(use --one-device to run the {N} shards on one GPU)")
    name, n_arg, topology, algorithm, window = workload(args, N)
    progress(0, f"{name}: {n_arg} {topology} {algorithm} over {N} shards "
                f"({'one device' if args.one_device else f'{N} devices'}, library multi-GPU engine)")
    base = base_line(args, 0, n_arg, topology, algorithm, window, ndev)
    cap = window if window else 1 << 40
    eng = Simulator(n_arg, topology, algorithm, seed=args.seed, device=0, num_gpus=N,
                    one_device=args.one_device, kernel_timing=not args.no_kernel_timing)
    bounds = sharded.partition(n_arg, topology, N)
    own = bounds[1] - bounds[0]
    progress(0, f"group ready ({eng.actors} actors, {own} on rank 0, {eng.layout.device_bytes / 2**30:.1f} GiB)")

    def sync_all():
        for d in range(1 if args.one_device else N):
            torch.cuda.synchronize(d)

    for _ in range(args.warmup):
        eng.reset()
        eng.step(cap)
    eng.kernel_stats(reset=True)
    rounds_total, converged = 0, True
    sync_all()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        eng.reset()
        st = eng.step(cap)
        rounds_total += int(st.round)
        converged &= bool(st.converged)
    sync_all()
    elapsed = time.perf_counter() - t0
    progress(0, f"{args.steps} timed step(s): {elapsed * 1e3:.1f} ms")
    ks = eng.kernel_stats()
    per_rank = {"actors": own, "world": N, "kernel": ks["kernel"], "aux_kernel": ks["aux_kernel"],
                "sampled_rounds": ks["launches"]}
    if args.one_device:
        # rank 0's hipEvents sit on a stream that shares the one device with every other shard's
        # kernels, so they bracket the other shards' work too: not a per-rank time
        per_rank.update(round_kernel_ms_device_shared=ks["avg_ms"], aux_kernel_ms_device_shared=ks["aux_avg_ms"],
                        timing_note="--one-device: rank 0's events bracket all shards' kernels on the shared "
                                    "device; per-rank kernel times come from a kernel trace "
                                    "(tools/shard_loopback_prof.py)")
    else:
        per_rank.update(round_kernel_ms=ks["avg_ms"], aux_kernel_ms=ks["aux_avg_ms"])
    transport = ("device copies on one GPU (GP_FLAG_ONE_DEVICE: the multi-GPU code path, no RCCL)"
                 if args.one_device else "RCCL ncclCommInitAll + grouped ncclSend/ncclRecv")
    out = emit_line(args, name=name, n_arg=n_arg, topology=topology, algorithm=algorithm, window=window,
                    eng_actors=eng.actors, eng_nodes=eng.nodes, grid=int(eng.layout.grid), own=own, n_gpus=N,
                    updates=float(eng.actors) * rounds_total, elapsed=elapsed, rounds_total=rounds_total,
                    converged=converged,
                    parallelism=f"node-range shards x{N}, one process, library multi-GPU engine; exchange: {transport}",
                    ks=ks, extra={"per_rank": per_rank, "devices": 1 if args.one_device else N,
                                  "launch": "one process (gp_config.num_gpus)"})
    attach_base(out, base, out["value"], N)
    print(json.dumps(out), flush=True)
    eng.close()
    return out


def main(argv=None):
    args = parse(argv)
    import torch
    import torch.distributed as dist

    if args.gpus < 1:
        fail("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return main_group(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and args.gpus != 1:
        fail(f"--gpus {args.gpus} but WORLD_SIZE={world}")
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
    base = None
    if world > 1:  # rank 0 times the window on its GPU alone while the other ranks wait
        base = base_line(args, rank, n_arg, topology, algorithm, window, torch.cuda.device_count())
        dist.barrier()
    cap = window if window else 1 << 40
    timing = not args.no_kernel_timing
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
        sent, received = eng.bytes_per_round()
        per_rank = dict(timer.means(), actors=own, bytes_sent_per_round=sent, bytes_received_per_round=received,
                        world=world, pieces=eng.npieces)
    out = None
    if rank == 0:
        cpu = None
        # the oracle holds the whole graph in host memory and builds it serially: beyond ~2e8
        # nodes its setup alone outlasts a bounded sample, so C5 (1e9) reports none
        if world == 1 and not args.no_cpu_baseline and n_arg <= CPU_BASELINE_MAX_N:
            progress(rank, "CPU baseline sample")
            cpu = cpu_baseline(n_arg, topology, algorithm, args.seed, args.cpu_seconds, window)
            if not use_shards:  # the GPU over the same rounds, for a same-span ratio
                cpu["gpu_value_same_rounds"] = gpu_same_window(eng, cpu["rounds"])
                cpu["gpu_over_cpu_same_rounds"] = cpu["gpu_value_same_rounds"] / cpu["value"]
        par = f"node-range shards x{world}, RCCL all-to-all" if use_shards else "single"
        out = emit_line(args, name=name, n_arg=n_arg, topology=topology, algorithm=algorithm, window=window,
                        eng_actors=eng.actors, eng_nodes=eng.nodes, grid=int(eng.layout.grid), own=own,
                        n_gpus=world, updates=updates, elapsed=elapsed, rounds_total=rounds_total,
                        converged=converged, parallelism=par, ks=ks, cpu=cpu,
                        extra={"per_rank": per_rank} if per_rank else None)
        if world > 1:
            out["launch"] = "torch.distributed.run, one process per GPU"
            attach_base(out, base, out["value"], world)
        print(json.dumps(out), flush=True)
    eng.close()
    if use_shards:
        dist.destroy_process_group()
    return out


if __name__ == "__main__":
    main()

"""W shards of one graph on ONE GPU (loopback exchange): per-kernel cost of the shard round at a
realistic remote fraction (e.g. 8 ranks -> 7/8 of the extra links remote), for A/B builds, and the
per-round cost of a whole run (every rank's round + the chunk copies + every rank's unpack,
bracketed with hipEvents on the shards' stream) with the phases of the run marked.

    python3 tools/shard_loopback_prof.py --world 8 --n 80000000 --rounds 64
    python3 tools/shard_loopback_prof.py --world 8 --n 100000000 --series out.json   # to convergence

The ranks run one after another on one GPU, so a round's time / world is the cost of one
rank-round without RCCL.  The summary compares the rounds in which every actor still sends (before
the first convergence) with the rounds after 99% of the nodes have converged (the quiet tail).
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cop5615-gossip_protocol_amd"))

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=80_000_000)
ap.add_argument("--world", type=int, default=8)
ap.add_argument("--topology", default="Imp3D")
ap.add_argument("--algorithm", default="push-sum")
ap.add_argument("--rounds", type=int, default=None, help="default: to convergence")
ap.add_argument("--seed", type=int, default=1)
ap.add_argument("--series", default=None, help="write the per-round series (JSON) here")
ap.add_argument("--no-pieces", action="store_true", help="one piece per round (no exchange overlap)")
ap.add_argument("--force-pieces", action="store_true", help="4 pieces at any size (the library's test hook)")
ap.add_argument("--rank0-events", action="store_true",
                help="also bracket rank 0's own round and unpack with events (each record stalls the queue "
                     "for a few microseconds, inside the phases the other figures time)")
ap.add_argument("--spin-us", type=float, default=0.0,
                help="a GPU spin of this many microseconds before every round, outside the timed events: "
                     "one host issues all W ranks' launches and copies here, and without a lead the GPU "
                     "waits for it in the short tail rounds (a node's host issues one rank's, batches ahead)")
a = ap.parse_args()

import torch  # noqa: E402

from gossip_amd import sharded  # noqa: E402

torch.cuda.set_device(0)
shards = [sharded.HipShard(a.n, a.topology, a.algorithm, rank=r, world=a.world, seed=a.seed, kernel_timing=True,
                           pieces=not a.no_pieces, force_pieces=a.force_pieces) for r in range(a.world)]
pieces_per_round = []
warmup_pieces = shards[0].npieces
nodes = shards[0].nodes
sharded.run_local(shards, max_rounds=8)  # warm-up (module load, first touches)
for e in shards:
    e.reset()
    e.kernel_stats(reset=True)
torch.cuda.synchronize()
cap = a.rounds if a.rounds else 1 << 40
t = sharded.LoopbackTransport()
events = []
sts = [e.sync() for e in shards]
send_bytes = [(0, shards[0].bytes_per_round()[0])]
round_bytes = []  # rank 0's send bytes per round (full gossip plans every round)
max_batch = sharded._max_batch(shards[0], 64)
batch = min(8, max_batch)
spin_cycles = 0
if a.spin_us > 0:  # calibrate torch.cuda._sleep's cycles against hipEvents
    c0 = 1 << 20
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda._sleep(c0)
    e0.record()
    torch.cuda._sleep(c0)
    e1.record()
    e1.synchronize()
    spin_cycles = int(c0 * a.spin_us / (e0.elapsed_time(e1) * 1e3))
t0 = time.perf_counter()
while not sts[0].converged and sts[0].round < cap:
    for _ in range(min(batch, cap - int(sts[0].round))):
        # the whole round on the shards' stream: every rank's round kernels and passes (in pieces:
        # each piece's chunk copies on the transport's own stream, overlapping the next piece), what
        # is left of the copies after the last piece (joined), every rank's unpack
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(6)]
        if spin_cycles:
            torch.cuda._sleep(spin_cycles)
        ev[0].record()
        K = shards[0].npieces  # (pieces until half the nodes have converged, one after)
        pieces_per_round.append(K)
        r0 = a.rank0_events and K == 1  # (ev[4], ev[5]: rank 0's own round and unpack, as round 4 timed them)
        if K == 1:
            for i, e in enumerate(shards):
                e.round()
                if i == 0 and r0:
                    ev[4].record()
            ev[1].record()
            t.exchange_all(shards)
        else:
            for i in range(K):  # (piece i's copies issued after piece i+1's kernels: sharded.run_local)
                for e in shards:
                    e.round_piece(i)
                t.piece_done(i)
                if i:
                    t.exchange_piece_all(shards, i - 1)
            ev[1].record()
            t.exchange_piece_all(shards, K - 1)
            t.join()
        round_bytes.append(shards[0].bytes_per_round()[0])  # rank 0's chunks of this round
        ev[2].record()
        for i, e in enumerate(shards):
            e.deliver()
            if i == 0 and r0:
                ev[5].record()
        ev[3].record()
        events.append((ev, K if r0 or K > 1 else 0))
    before = int(sts[0].completed)
    sts = [e.sync() for e in shards]
    assert len({(int(s.round), int(s.completed), int(s.converged)) for s in sts}) == 1, "shards disagree"
    send_bytes.append((int(sts[0].round), shards[0].bytes_per_round()[0]))  # rank 0's plan from here on
    batch = sharded._next_batch(batch, max_batch, nodes, before, int(sts[0].completed))  # the product loop's schedule
torch.cuda.synchronize()
el = time.perf_counter() - t0
rounds = int(sts[0].round)
trace = [int(x) for x in shards[0].read_trace()]
# gossip's F(k) applies round k - 1: one launch more than rounds
launches = rounds + (1 if a.algorithm == "gossip" else 0)
nl = min(launches, len(events))
per_round = [events[i][0][0].elapsed_time(events[i][0][3]) for i in range(nl)]
# the phases of a round on the shards' stream (all ranks): the round kernels and passes (in pieces
# the copies of all but the last piece run beside them), the copies not hidden, the unpacks
compute = [events[i][0][0].elapsed_time(events[i][0][1]) for i in range(nl)]
copies = [events[i][0][1].elapsed_time(events[i][0][2]) for i in range(nl)]
unpack = [events[i][0][2].elapsed_time(events[i][0][3]) for i in range(nl)]
# rank 0's own work (its round kernels + passes, its unpack; one-piece rounds only): what one GPU of
# a real node would spend beside its all-to-all
rank0 = [(events[i][0][0].elapsed_time(events[i][0][4]) + events[i][0][2].elapsed_time(events[i][0][5]))
         if events[i][1] == 1 else None for i in range(nl)]
# every rank's round kernels and unpacks without the copies, per rank (hipEvents around whole phases)
kern = [compute[i] + unpack[i] for i in range(nl)]
ks = shards[0].kernel_stats()


def mean(xs):
    return statistics.fmean(xs) if xs else None


# round r is "dense" while fewer than 1% of the nodes had converged after round r - 1 (nearly every
# actor sends), "tail" once 99% had
prev = [0] + trace[:-1]
dense_r = [r for r in range(nl) if r < len(prev) and prev[r] * 100 < nodes]
tail_r = [r for r in range(nl) if r < len(prev) and prev[r] * 100 >= 99 * nodes]


def phase(xs, rs, div=1.0):
    v = [xs[r] for r in rs if xs[r] is not None]
    return mean(v) / div if v else None


summary = {
    "workload": f"{a.n} {a.topology} {a.algorithm}", "world": a.world, "rounds": rounds,
    "converged": bool(sts[0].converged), "host_ms": el * 1e3,
    "round_ms_sum": sum(per_round),
    "rounds_dense_lt1pct": len(dense_r), "rounds_tail_99pct": len(tail_r),
    # one round of all ranks / world (rank kernels serialised + every chunk copy)
    "rank_round_ms_dense": phase(per_round, dense_r, a.world),
    "rank_round_ms_tail": phase(per_round, tail_r, a.world),
    "tail_over_dense": phase(per_round, tail_r) / phase(per_round, dense_r) if dense_r and tail_r else None,
    "kernels_ms_dense": phase(kern, dense_r, a.world), "kernels_ms_tail": phase(kern, tail_r, a.world),
    "kernels_tail_over_dense": phase(kern, tail_r) / phase(kern, dense_r) if dense_r and tail_r else None,
    # per rank-round (all ranks / world): round kernels and passes, the copies left exposed after
    # the last piece (in pieces; else all of them), the unpack
    "pieces_first": pieces_per_round[0] if pieces_per_round else None,
    "rounds_in_pieces": sum(1 for k in pieces_per_round if k > 1),
    "compute_ms_dense": phase(compute, dense_r, a.world), "exposed_copies_ms_dense": phase(copies, dense_r, a.world),
    "unpack_ms_dense": phase(unpack, dense_r, a.world),
    "compute_ms_tail": phase(compute, tail_r, a.world), "exposed_copies_ms_tail": phase(copies, tail_r, a.world),
    "unpack_ms_tail": phase(unpack, tail_r, a.world),
    # rank 0's own round + unpack by hipEvents (one-piece rounds)
    "spin_us": a.spin_us,
    "rank0_ms_dense": phase(rank0, dense_r), "rank0_ms_tail": phase(rank0, tail_r),
    "rank0_tail_over_dense": (phase(rank0, tail_r) / phase(rank0, dense_r)
                              if phase(rank0, dense_r) and phase(rank0, tail_r) else None),
    "rank0_kernel": ks["kernel"], "rank0_kernel_avg_ms": ks["avg_ms"], "rank0_aux": ks["aux_kernel"],
    "rank0_aux_avg_ms": ks["aux_avg_ms"], "rank0_work_per_launch": ks["work_per_launch"],
    "rank0_actors": shards[0].hi - shards[0].lo,
    "send_bytes_rank0_full_plan": int(shards[0].shard.send_total),
    "send_bytes_rank0_run": sum(round_bytes),  # every round packed, replays included
    "send_bytes_rank0_if_full_plan": len(round_bytes) * int(shards[0].shard.send_total),
    "send_bytes_rank0_least": min(b for _, b in send_bytes),
    "shard_stats_rank0": shards[0].shard_stats(),
    "note": "all ranks serialised on one GPU; exchange = device copies (no RCCL); rank-round = round / world",
}
print(json.dumps(summary, indent=1), flush=True)
if a.series:
    with open(a.series, "w") as f:
        json.dump(dict(summary, per_round_ms=[round(x, 4) for x in per_round],
                       compute_ms=[round(x, 4) for x in compute], copies_ms=[round(x, 4) for x in copies],
                       rank0_ms=[None if x is None else round(x, 4) for x in rank0],
                       unpack_ms=[round(x, 4) for x in unpack],
                       send_bytes=send_bytes, round_bytes=round_bytes, trace=trace,
                       pieces_per_round=pieces_per_round, warmup_pieces=warmup_pieces), f)
for e in shards:
    e.close()

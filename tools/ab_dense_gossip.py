"""the sparse receipt exchange of full gossip against a dense u8 histogram
reduce-scatter, on 8 loopback shards of one graph on one GPU.

    python tools/ab_dense_gossip.py [--n 100000000] [--world 8]

Sparse (the engine): every round each rank sends, to each peer, the target ids of the
receipts its chains produced for that peer's actors (4 B each, sub-segmented).
The script runs the real shards (gp_shard_*) through the loopback transport, reads every chunk
header to count the entries actually sent, and times each round's phases with events.

Dense: each rank would instead build a histogram of its receipts over ALL actors (1 B per
actor, assuming no target receives more than 255 of them from one rank) and reduce-scatter it:
every rank sends (world-1)/world of the histogram each round whatever the activity.  Timed here
on the same receipts: torch.bincount of each rank's targets (the histogram), the u8 cast, and
the loopback reduce-scatter (copies of the world slices + the sum), on the same GPU.

Prints one JSON line: per-round bytes and times of both, and the totals to convergence.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cop5615-gossip_protocol_amd"))

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=100_000_000)
ap.add_argument("--world", type=int, default=8)
ap.add_argument("--seed", type=int, default=1)
args = ap.parse_args()

import torch  # noqa: E402

from gossip_amd import sharded  # noqa: E402

W = args.world
engines = [sharded.HipShard(args.n, "full", "gossip", rank=r, world=W, seed=args.seed) for r in range(W)]
A = engines[0].actors
bounds = [e.lo for e in engines] + [engines[-1].hi]
so = [np.concatenate([[0], np.cumsum(e.send_splits)]) for e in engines]
t = sharded.LoopbackTransport()
ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731

rounds = []
st = [e.sync() for e in engines]
while not st[0].converged:
    e0, e1, e2, e3 = ev(), ev(), ev(), ev()
    e0.record()
    for e in engines:
        e.round()
    e1.record()
    t.exchange_all(engines)
    e2.record()
    for e in engines:
        e.deliver()
    e3.record()
    # entries each rank sent this round (chunk headers: u32 nlinks[16] at byte 16)
    entries = 0
    for p, e in enumerate(engines):
        buf = e.send_buf
        for q in range(W):
            if q == p or not e.send_splits[q]:
                continue
            hdr = buf[so[p][q]:so[p][q] + 256].cpu().numpy()
            nl = hdr[16:80].view(np.uint32)
            entries += int(nl.sum())
    torch.cuda.synchronize()
    sparse_ms = e1.elapsed_time(e2) + e2.elapsed_time(e3)  # exchange + unpack (the round kernels are common)
    # dense: per rank a u8 histogram over all actors of its receipts, then the reduce-scatter
    gen = torch.Generator(device="cuda").manual_seed(len(rounds))
    per_rank = max(1, entries // W)  # this round's receipts per rank (the sparse engine's count)
    d0, d1, d2 = ev(), ev(), ev()
    d0.record()
    hists = []
    for p in range(W):
        tg = torch.randint(0, A, (per_rank,), device="cuda", generator=gen)
        hists.append(torch.bincount(tg, minlength=A).to(torch.uint8))
    d1.record()
    for q in range(W):
        lo, hi = bounds[q], bounds[q + 1]
        acc = torch.zeros(hi - lo, dtype=torch.int32, device="cuda")
        for p in range(W):
            acc += hists[p][lo:hi].to(torch.int32)  # the slice rank p would send to rank q
    d2.record()
    torch.cuda.synchronize()
    rounds.append({"entries": entries, "sparse_bytes": entries * 4, "sparse_ms": sparse_ms,
                   "dense_bytes": A * (W - 1), "dense_hist_ms": d0.elapsed_time(d1),
                   "dense_rs_ms": d1.elapsed_time(d2)})
    st = [e.sync() for e in engines]
    del hists

tot = {k: sum(r[k] for r in rounds) for k in rounds[0]}
print(json.dumps({"n": args.n, "actors": A, "world": W, "rounds": len(rounds), "per_round": rounds, "total": tot}))

"""Multi-rank path on CPU: the product's shard host loop (gossip_amd.sharded.run) and its
torch.distributed transport, over gloo with world_size 2, 3 and 8, driving the CPU oracle's shard
engine (oracle.OracleShard).  Each rank owns the node range gp_partition gives it (whole
z-planes for Imp3D/3D); the job must reproduce the single-process oracle bit for bit —
completion trace, convergence round and every actor's state."""
from __future__ import annotations

import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CASES = [
    # (n_arg, topology, algorithm, seed, round cap)
    (1000, "Imp3D", "push-sum", 1, 4000),
    (200, "3D", "push-sum", 3, 4000),
    (200, "line", "push-sum", 2, 300),
    (50, "2D", "push-sum", 3, 400),
    (1000, "full", "gossip", 1, 4000),
    (1000, "Imp3D", "gossip", 3, 4000),
    (200, "line", "gossip", 3, 20000),
    (64, "2D", "gossip", 2, 20000),
    (200, "3D", "gossip", 1, 4000),
]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class PiecedOracle:
    """The oracle's shard engine behind the piece API of HipShard (npieces, round_piece, piece_plans):
    each round's chunk p -> q is cut into K byte ranges, laid out piece-major as the library lays out
    its pieces, and moved by K all-to-alls (TorchTransport.exchange_piece / join), which the host loop
    (sharded.run) issues one per piece.  Checks the piece transport and loop on CPU."""

    def __init__(self, eng, K):
        import torch

        self.e, self.npieces, self.layout = eng, K, eng.layout
        so = np.concatenate([[0], np.cumsum(eng.send_splits)])
        ro = np.concatenate([[0], np.cumsum(eng.recv_splits)])
        self.piece_plans, self.smap, self.rmap = [], [], []
        sb = rb = 0
        for i in range(K):
            ss = [n * (i + 1) // K - n * i // K for n in eng.send_splits]
            rs = [n * (i + 1) // K - n * i // K for n in eng.recv_splits]
            self.piece_plans.append((ss, rs, sb, rb))
            for q, n in enumerate(eng.send_splits):
                self.smap.append((sb, int(so[q]) + n * i // K, ss[q]))
                sb += ss[q]
            for q, n in enumerate(eng.recv_splits):
                self.rmap.append((rb, int(ro[q]) + n * i // K, rs[q]))
                rb += rs[q]
        self.send_buf = torch.zeros(sb, dtype=torch.uint8)
        self.recv_buf = torch.zeros(rb, dtype=torch.uint8)

    def round_piece(self, i):
        if i == 0:  # the oracle computes the round whole; piece i only moves bytes
            self.e.round()
            for dst, src, n in self.smap:
                self.send_buf[dst:dst + n] = self.e.send_buf[src:src + n]

    def deliver(self):
        for src, dst, n in self.rmap:
            self.e.recv_buf[dst:dst + n] = self.recv_buf[src:src + n]
        self.e.deliver()

    def sync(self):
        return self.e.sync()

    def __getattr__(self, name):  # read_*, lo, hi, ...
        return getattr(self.e, name)


def _worker(rank, world, port, case, bounds, q, pieces=1):
    for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "cop5615-gossip_protocol_amd")):
        sys.path.insert(0, p)
    import torch.distributed as dist

    import oracle
    from gossip_amd import sharded

    n, topo, algo, seed, cap = case
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        eng = oracle.OracleShard(n, topo, algo, rank=rank, world=world, bounds=bounds, seed=seed)
        if pieces > 1:
            eng = PiecedOracle(eng, pieces)
        st = sharded.run(eng, sharded.TorchTransport(), max_rounds=cap)
        state = eng.read_gossip() if algo == "gossip" else eng.read_pushsum()
        sums = None
        if algo == "push-sum":  # global mass = sum over ranks of held + in-flight
            import torch
            t = torch.tensor([st.sum_s, st.sum_w], dtype=torch.float64)
            dist.all_reduce(t)
            sums = t.tolist()
        q.put((rank, int(st.round), int(st.completed), int(st.converged), eng.read_trace(),
               [np.asarray(a) for a in state], sums))
    finally:
        dist.destroy_process_group()


def _run_job(case, world, bounds, pieces=1):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, case, bounds, q, pieces)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(out, key=lambda x: x[0])


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("case", CASES, ids=lambda c: f"{c[2]}-{c[1]}-{c[0]}")
def test_sharded_matches_single_process(case, world, pieces=1):
    import oracle
    from gossip_amd import sharded

    n, topo, algo, seed, cap = case
    bounds = sharded.partition(n, topo, world)
    ref = oracle.OracleSim(n, topo, algo, seed=seed)
    rs = ref.step(cap)
    ref_state = ref.read_gossip() if algo == "gossip" else ref.read_pushsum()
    ref_trace = ref.read_trace()
    out = _run_job(case, world, bounds, pieces)
    for rank, rnd, comp, conv, trace, state, sums in out:
        assert (rnd, comp, conv) == (rs.round, rs.completed, rs.converged), (rank, rnd, rs.round)
        np.testing.assert_array_equal(trace, ref_trace)
        lo, hi = bounds[rank], bounds[rank + 1]
        for got, want in zip(state, ref_state):
            np.testing.assert_array_equal(got, want[lo:hi])  # bit-exact, fp64 included
        if sums is not None:  # conservation: sum s = sum of ids, sum w = participants
            assert sums[1] == pytest.approx(ref.layout.participants, rel=1e-12)
            assert sums[0] == pytest.approx(rs.sum_s, rel=1e-12)
    ref.close()


@pytest.mark.parametrize("case", [(1000, "Imp3D", "push-sum", 1, 4000), (1000, "full", "gossip", 1, 4000)],
                         ids=lambda c: f"{c[2]}-{c[1]}-{c[0]}")
def test_sharded_world8(case):
    """The driver's rank count (8 processes over gloo): the same host loop and transport."""
    test_sharded_matches_single_process(case, 8)


@pytest.mark.parametrize("world,pieces", [(2, 4), (3, 3)])
@pytest.mark.parametrize("case", [(1000, "Imp3D", "push-sum", 1, 4000), (200, "line", "push-sum", 2, 300)],
                         ids=lambda c: f"{c[2]}-{c[1]}-{c[0]}")
def test_sharded_pieces_gloo(case, world, pieces):
    """A round in pieces through the product host loop: one asynchronous
    all-to-all per piece (TorchTransport.exchange_piece, joined before the unpack), bit-exact
    against one process."""
    test_sharded_matches_single_process(case, world, pieces)


def test_uneven_partition_gossip_full():
    """Any contiguous split gives the same run (here not the gp_partition one)."""
    import oracle

    case = (300, "full", "gossip", 2, 4000)
    bounds = [0, 17, 301]
    ref = oracle.OracleSim(300, "full", "gossip", seed=2)
    rs = ref.step(4000)
    cnt, flags = ref.read_gossip()
    out = _run_job(case, 2, bounds)
    for rank, rnd, comp, conv, trace, state, _ in out:
        assert (rnd, comp, conv) == (rs.round, rs.completed, rs.converged)
        lo, hi = bounds[rank], bounds[rank + 1]
        np.testing.assert_array_equal(state[0], cnt[lo:hi])
        np.testing.assert_array_equal(state[1], flags[lo:hi])


def test_partition_rules():
    from gossip_amd import sharded

    # Imp3D 10M: nodes 9,938,375, G = 239, plane 57,121, 174 planes
    b = sharded.partition(10_000_000, "Imp3D", 8)
    assert b[0] == 0 and b[-1] == 9_938_376 and len(b) == 9
    assert all(x % 57_121 == 0 for x in b[1:-1])
    assert all(b[i] < b[i + 1] for i in range(8))
    b = sharded.partition(1000, "line", 3)
    assert b == [0, 333, 667, 1001]
    from gossip_amd import GossipError
    with pytest.raises(GossipError):
        sharded.partition(20, "Imp3D", 8)  # 2 z-planes cannot feed 8 ranks
    with pytest.raises(GossipError):
        sharded.partition(1000, "Imp3D", 17)  # more ranks than the exchange supports


def _sweep_cases(count=8, seed=12):
    """Seeded random (n, topology, algorithm, seed) draws over 2..5 ranks (no push-sum on
    "full": single-GPU only); sizes log-uniform over 64..3000."""
    rng = np.random.default_rng(seed)
    topos = ["2D", "3D", "Imp3D", "full", "line"]
    out = []
    while len(out) < count:
        n = int(np.exp(rng.uniform(np.log(64), np.log(3000))))
        topo, algo = topos[rng.integers(len(topos))], ("gossip", "push-sum")[rng.integers(2)]
        world = int(rng.integers(2, 6))
        if topo == "full" and algo == "push-sum":
            continue
        out.append(((n, topo, algo, int(rng.integers(1, 1 << 30)), 3000), world))
    return out


@pytest.mark.parametrize("case,world", _sweep_cases(), ids=lambda c: str(c))
def test_sharded_random_sweep(case, world):
    """Random configurations through the product host loop and gloo transport, bit-exact
    against one process."""
    from gossip_amd import GossipError, sharded

    try:
        sharded.partition(case[0], case[1], world)
    except GossipError as e:
        if "cannot be split" not in str(e):
            raise
        pytest.skip(str(e))
    test_sharded_matches_single_process(case, world)


@pytest.mark.parametrize("world,case", [(2, (1000, "Imp3D", "push-sum", 1, 0)), (3, (1000, "full", "gossip", 2, 0))],
                         ids=lambda c: str(c))
def test_dist_shard_job_script_gloo(world, case):
    """The launcher and rank script of the cross-device nccl test (tests/dist_shard_job.py under
    torch.distributed.run, test_gpu_multidevice.py) on CPU: gloo + the oracle's shard engine, the
    joined rank parts bit-exact against one process."""
    import oracle
    from helpers import join_parts, run_dist_job, state_arrays

    n, topo, algo, seed, cap = case
    ref = oracle.OracleSim(n, topo, algo, seed=seed)
    rs = ref.step()
    want = state_arrays(ref, algo)
    parts = run_dist_job(world, "gloo", n, topo, algo, seed, cap, 300)
    for p in parts:
        assert tuple(int(x) for x in p["status"]) == (rs.round, rs.completed, rs.converged)
        np.testing.assert_array_equal(p["trace"], ref.read_trace())
    got = join_parts(parts, list(want))
    for k in want:
        np.testing.assert_array_equal(got[k], want[k])
    ref.close()


def test_batch_schedule_restarts_at_half_reported():
    """The host loop's batches double up to the cap and start again from 8 rounds at the sync
    where the run passes half of the nodes reported (the activity tiers' first decision)."""
    from gossip_amd.sharded import _next_batch
    assert _next_batch(8, 64, 1000, 0, 10) == 16
    assert _next_batch(64, 64, 1000, 0, 10) == 64
    assert _next_batch(32, 64, 1000, 499, 500) == 8
    assert _next_batch(32, 64, 1000, 100, 999) == 8
    assert _next_batch(8, 64, 1000, 500, 600) == 16  # already past half: no restart

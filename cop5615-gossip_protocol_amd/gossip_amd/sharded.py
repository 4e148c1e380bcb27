"""Multi-GPU host: one graph split into node-range shards, one process (or handle) per GPU.

The reference has no distributed mode: its only parallelism is the Akka dispatcher running
the actors on the .NET thread pool (program.fs:23), and the ParentActor counts reports until
`AllNodes` (program.fs:44-63).  Here every rank owns a contiguous actor range
(``gp_partition``: whole z-planes for Imp3D/3D) and one round is

    engine.round()          # F(k) on this rank's actors + pack what other ranks need
    transport.exchange()    # ONE all-to-all (RCCL over xGMI); chunk sizes change only at a sync
    engine.deliver()        # unpack: halo faces, cross-shard link messages, global count

or, for a large push-sum shard, the same round in pieces: the all-to-all of piece i
runs (asynchronously, on the transport's own stream) while piece i+1 is computed, and the unpack
waits for the last one.

with everything enqueued on the engine's HIP stream — the host only waits every few rounds
(``engine.sync()``) to learn whether the global completion count reached `nodes`.  At that sync
a push-sum shard also sizes the next batch's chunks from the activity of the last one (activity
tiers, gp_shard_plan), and may rewind to a restore point if a reduced chunk overflowed: the host
loop just runs on from the round the sync reports.

Engines: :class:`HipShard` (libgossip_hip.so on a GPU — the product) and, in the tests,
``oracle.OracleShard`` (the CPU checker).  Transports: :class:`TorchTransport`
(torch.distributed all_to_all_single: RCCL for CUDA tensors, gloo for CPU tensors) and
:class:`LoopbackTransport` (several shards inside one process).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _abi


def partition(n_arg: int, topology: str, world: int):
    """Actor bounds of every rank (gp_partition): list of world+1 ints."""
    b = np.zeros(world + 1, np.int64)
    _abi.check(_abi.load().gp_partition(n_arg, _abi.TOPOLOGIES[topology], world,
                                        b.ctypes.data_as(C.c_void_p)))
    return [int(x) for x in b]


class HipShard:
    """Rank `rank` of `world` on HIP device `device` (gp_create_shard)."""

    def __init__(self, n_arg: int, topology: str, algorithm: str, *, rank: int, world: int, seed: int = 1,
                 device: int = 0, stream: int | None = None, kernel_timing: bool = False, delta: float = 1e-10,
                 gossip_threshold: int = 10, term_init: int = 1, term_limit: int = 3, quiet_waves: bool = False,
                 full_plan: bool = False, tight_tiers: bool = False, pieces: bool = True,
                 force_pieces: bool = False, force_bins: bool = False):
        """quiet_waves: the push-sum quiet-tail walk at any shard size (a test hook; on by default
        for shards of 2^20 actors or more).  full_plan: no activity tiers (every round ships the
        all-sending capacity); tight_tiers: tiers with no headroom and frequent replays (a test
        hook).  pieces: exchange a push-sum round piece by piece (the library picks 4 pieces from
        2^25 actors per rank until half the nodes have converged, else 1); force_pieces: 4 pieces
        at any size (a test hook).  force_bins: full gossip sends its receipts in bins in every round
        past the ramp's lists (by default the receipt wave only; a test hook)."""
        import torch

        if topology not in _abi.TOPOLOGIES:
            raise ValueError(f"unknown topology {topology!r} (case-sensitive: {list(_abi.TOPOLOGIES)})")
        if algorithm not in _abi.ALGOS:
            raise ValueError("Invalid:Please enter a proper protocol or topology")
        self.lib = _abi.load()
        # torch's current stream by default, so the exchange (RCCL / copies) is ordered with the
        # kernels; its handle may be 0 (the null stream), hence FLAG_USE_STREAM
        flags = (_abi.FLAG_KERNEL_TIMING if kernel_timing else 0) | _abi.FLAG_USE_STREAM
        flags |= _abi.FLAG_QUIET_WAVES if quiet_waves else 0
        flags |= (_abi.FLAG_FULL_PLAN if full_plan else 0) | (_abi.FLAG_TIGHT_TIERS if tight_tiers else 0)
        flags |= (_abi.FLAG_PIECES if pieces or force_pieces else 0) | (_abi.FLAG_FORCE_PIECES if force_pieces else 0)
        flags |= _abi.FLAG_GOSSIP_TALLY if force_bins else 0
        if stream is None:
            stream = torch.cuda.current_stream(device).cuda_stream
        self.cfg = _abi.Config(n_arg, _abi.TOPOLOGIES[topology], _abi.ALGOS[algorithm], seed, delta,
                               gossip_threshold, term_init, term_limit, device, flags, 0, stream)
        self.layout = _abi.Layout()
        self.shard = _abi.ShardLayout()
        h = C.c_void_p()
        _abi.check(self.lib.gp_create_shard(C.byref(self.cfg), rank, world, C.byref(self.layout),
                                            C.byref(self.shard), C.byref(h)))
        self.h = h
        self.rank, self.world = rank, world
        self.topology, self.algorithm = topology, algorithm
        self.lo, self.hi = int(self.shard.lo), int(self.shard.hi)
        self.npieces = int(self.lib.gp_shard_pieces(self.h))
        # full gossip sizes every round's chunks from the last round before a sync:
        # its host loop syncs every 4 rounds, so the plans follow the run's activity (its receipts
        # thin out by a third or more per round once targets report)
        self.max_batch = 4 if (topology == "full" and algorithm == "gossip" and world > 1) else None
        self._plan()
        dev = torch.device("cuda", device)
        # buffers for the full plan (the first one); the caching allocator hands out 512-byte
        # aligned blocks (the ABI needs 256)
        st, rt = int(self.shard.send_total), int(self.shard.recv_total)
        self.send_buf = torch.zeros(max(1, st), dtype=torch.uint8, device=dev)[:st]
        # two receive buffers, one per round parity: a push-sum round reads the previous round's remote
        # messages where they arrived, and in pieces the next exchange overlaps it
        self._recv = [torch.zeros(max(1, rt), dtype=torch.uint8, device=dev)[:rt] for _ in range(2)]
        self._ri = 0
        self.status = _abi.Status()

    @property
    def recv_buf(self):
        """The receive buffer of the round in progress (the exchange writes it, deliver() reads it)."""
        return self._recv[self._ri]

    def _plan(self):
        """The next round's per-peer chunk sizes (gp_shard_plan): they follow the activity of the
        run (push-sum: per batch; full gossip: per round), so they are re-read after every round
        and sync.  In pieces: piece_plans[i] = (send splits, recv splits, send offset, recv offset)
        of piece i (gp_shard_plan_piece)."""
        if not hasattr(self, "_sb"):
            self._sb = np.zeros(self.world, np.int64)
            self._rb = np.zeros(self.world, np.int64)
            self._ob = np.zeros(2, np.int64)
            self._sbp = self._sb.ctypes.data_as(C.c_void_p)
            self._rbp = self._rb.ctypes.data_as(C.c_void_p)
            self._obp = self._ob.ctypes.data_as(C.c_void_p)
        # pieces until half the nodes have converged, one piece after (the library decides at a sync)
        self.npieces = int(self.lib.gp_shard_pieces(self.h))
        if self.npieces == 1:
            _abi.check(self.lib.gp_shard_plan(self.h, self._sbp, self._rbp))
            self.send_splits, self.recv_splits = self._sb.tolist(), self._rb.tolist()
            self.piece_plans = [(self.send_splits, self.recv_splits, 0, 0)]
            return
        self.piece_plans = []
        for i in range(self.npieces):
            _abi.check(self.lib.gp_shard_plan_piece(self.h, i, self._sbp, self._rbp, self._obp))
            self.piece_plans.append((self._sb.tolist(), self._rb.tolist(), int(self._ob[0]), int(self._ob[1])))
        self.send_splits = self.recv_splits = None  # per piece only

    def bytes_per_round(self):
        """(send, receive) bytes of the current plan's whole round (every piece)."""
        return (sum(sum(p[0]) for p in self.piece_plans), sum(sum(p[1]) for p in self.piece_plans))

    def shard_stats(self):
        s = _abi.ShardStats()
        _abi.check(self.lib.gp_shard_stats(self.h, C.byref(s)))
        return {"plan_changes": s.plan_changes, "restores": s.restores, "send_bytes": s.send_bytes,
                "recv_bytes": s.recv_bytes, "restore_round": s.restore_round, "bytes_sent": s.bytes_sent,
                "list_rounds": s.list_rounds, "bin_rounds": s.bin_rounds}

    @property
    def nodes(self) -> int:
        return int(self.layout.nodes)

    @property
    def actors(self) -> int:
        return int(self.layout.actors)

    def round(self):
        _abi.check(self.lib.gp_shard_round(self.h, C.c_void_p(self.send_buf.data_ptr())))
        self._plan()  # this round's chunk sizes (the exchange that follows moves them)

    def round_piece(self, i: int):
        """Piece i of the round (in order); its exchange may start at once (piece_plans[i])."""
        _abi.check(self.lib.gp_shard_round_piece(self.h, C.c_void_p(self.send_buf.data_ptr()), i))

    def deliver(self):
        _abi.check(self.lib.gp_shard_deliver(self.h, C.c_void_p(self.recv_buf.data_ptr())))
        self._ri ^= 1

    def sync(self):
        _abi.check(self.lib.gp_shard_sync(self.h, C.byref(self.status)))
        self._plan()
        return self.status

    def reset(self):
        _abi.check(self.lib.gp_reset(self.h))
        self.status = _abi.Status()
        self._plan()

    # read-back of this rank's actors [lo, hi) (global ids)
    def read_gossip(self):
        n = self.hi - self.lo
        cnt = np.zeros(n, np.uint32)
        flags = np.zeros(n, np.uint8)
        _abi.check(self.lib.gp_read_gossip(self.h, self.lo, n, cnt.ctypes.data_as(C.c_void_p),
                                           flags.ctypes.data_as(C.c_void_p)))
        return cnt, flags

    def read_pushsum(self):
        n = self.hi - self.lo
        S = np.zeros(n, np.float64)
        W = np.zeros(n, np.float64)
        flags = np.zeros(n, np.uint8)
        _abi.check(self.lib.gp_read_pushsum(self.h, self.lo, n, S.ctypes.data_as(C.c_void_p),
                                            W.ctypes.data_as(C.c_void_p), flags.ctypes.data_as(C.c_void_p)))
        return S, W, flags

    def read_messages(self):
        """Push-sum messages this rank's actors emitted in the last round: dst, s, w."""
        n = self.hi - self.lo
        d = np.zeros(n, np.uint32)
        s = np.zeros(n, np.float64)
        w = np.zeros(n, np.float64)
        _abi.check(self.lib.gp_read_messages(self.h, self.lo, n, d.ctypes.data_as(C.c_void_p),
                                             s.ctypes.data_as(C.c_void_p), w.ctypes.data_as(C.c_void_p)))
        return d, s, w

    def read_trace(self):
        r = int(self.status.round)
        out = np.zeros(r, np.int64)
        if r:
            _abi.check(self.lib.gp_read_trace(self.h, 0, r, out.ctypes.data_as(C.c_void_p)))
        return out

    def kernel_stats(self, reset: bool = False):
        ks = _abi.KStats()
        _abi.check(self.lib.gp_kernel_stats(self.h, C.byref(ks), 1 if reset else 0))
        return {"launches": ks.launches, "total_ms": ks.total_ms, "avg_ms": ks.avg_ms,
                "bytes_per_launch": ks.bytes_per_launch, "kernel": ks.kernel.decode(),
                "aux_avg_ms": ks.aux_avg_ms, "aux_kernel": ks.aux_kernel.decode(),
                "work_per_launch": ks.work_per_launch}

    def close(self):
        if getattr(self, "h", None):
            self.lib.gp_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class TorchTransport:
    """The per-round exchange as one torch.distributed all_to_all_single: RCCL over xGMI for
    device buffers (backend "nccl" on ROCm), gloo for CPU buffers.  Sizes change only at a sync
    (the engine's plan), so there is no count exchange and no host synchronisation inside a
    round."""

    def __init__(self, group=None):
        import torch.distributed as dist

        self.dist = dist
        self.group = group

    def exchange(self, eng):
        # the current plan's chunks are packed from offset 0 (a prefix of the full-plan buffers)
        ns, nr = sum(eng.send_splits), sum(eng.recv_splits)
        self.dist.all_to_all_single(eng.recv_buf[:nr], eng.send_buf[:ns], eng.recv_splits, eng.send_splits,
                                    group=self.group)

    def exchange_piece(self, eng, i):
        """Piece i's all-to-all, asynchronous: it waits for the kernels enqueued so far (piece i's)
        and runs on the process group's stream while the next piece is computed; join() makes the
        engine's stream wait for it."""
        ss, rs, so, ro = eng.piece_plans[i]
        return self.dist.all_to_all_single(eng.recv_buf[ro:ro + sum(rs)], eng.send_buf[so:so + sum(ss)], rs, ss,
                                           group=self.group, async_op=True)

    def join(self, works):
        for w in works:
            w.wait()


def _offsets(splits):
    return np.concatenate([[0], np.cumsum(splits)]).astype(np.int64)


class LoopbackTransport:
    """All shards live in this process (one GPU, or CPU): chunk p->q is copied from p's send
    buffer into q's receive buffer (stream-ordered device copies for HipShard).  In pieces the
    copies of piece i run on a stream of their own, after every shard's piece i (piece_done), while
    the shards compute piece i+1 (join: the engines' stream waits for the copies).  The host issues
    piece i's copies after piece i+1's kernels (run_local): one process issues every rank's copies,
    and issued first they kept the kernels of piece i+1 waiting for the host."""

    def __init__(self):
        self.stream = None
        self.done = {}

    def piece_done(self, i):
        """Every shard's piece i is enqueued on the current stream."""
        import torch

        self.done[i] = torch.cuda.Event()
        self.done[i].record()

    def exchange_piece_all(self, engines, i):
        import torch

        if self.stream is None:
            self.stream = torch.cuda.Stream()
        ev = self.done.pop(i, None)
        if ev is not None:
            self.stream.wait_event(ev)  # after every shard's piece i
        else:
            self.stream.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(self.stream):
            plans = [e.piece_plans[i] for e in engines]
            so = [_offsets(pl[0]) + pl[2] for pl in plans]
            ro = [_offsets(pl[1]) + pl[3] for pl in plans]
            for p, ep in enumerate(engines):
                for q, eq in enumerate(engines):
                    n = plans[p][0][q]
                    if p == q or n == 0:
                        continue
                    assert n == plans[q][1][p], (p, q, n, plans[q][1][p])
                    eq.recv_buf[ro[q][p]:ro[q][p] + n].copy_(ep.send_buf[so[p][q]:so[p][q] + n])

    def join(self):
        import torch

        if self.stream is not None:
            torch.cuda.current_stream().wait_stream(self.stream)

    def exchange_all(self, engines):
        so = [_offsets(e.send_splits) for e in engines]
        ro = [_offsets(e.recv_splits) for e in engines]
        for p, ep in enumerate(engines):
            for q, eq in enumerate(engines):
                n = ep.send_splits[q]
                if p == q or n == 0:
                    continue
                assert n == eq.recv_splits[p], (p, q, n, eq.recv_splits[p])
                eq.recv_buf[ro[q][p]:ro[q][p] + n].copy_(ep.send_buf[so[p][q]:so[p][q] + n])


class PhaseTimer:
    """Per-phase device time of one rank's rounds, from events on the stream the engine runs on
    (torch's current stream): every `every`-th round is bracketed as round (the round kernel, the
    link scatter, the halo and the chunk headers) | exchange (the all-to-all) | deliver (unpack)."""

    def __init__(self, every: int = 8):
        import torch

        self.torch = torch
        self.every = every
        self.pending = []
        self.n = 0
        self.ms = {"round": 0.0, "exchange": 0.0, "deliver": 0.0}
        self.count = 0

    def events(self):
        self.count += 1
        if (self.count - 1) % self.every:
            return None
        ev = [self.torch.cuda.Event(enable_timing=True) for _ in range(4)]
        self.pending.append(ev)
        return ev

    def collect(self):
        for ev in self.pending:
            ev[3].synchronize()
            for k, (a, b) in zip(("round", "exchange", "deliver"), zip(ev[:3], ev[1:])):
                self.ms[k] += a.elapsed_time(b)
            self.n += 1
        self.pending = []

    def means(self):
        return {k + "_ms": (v / self.n if self.n else None) for k, v in self.ms.items()}


def run(engine, transport, max_rounds: int = 1 << 40, batch: int = 8, max_batch: int = 64, timer=None):
    """Advance this rank until the GLOBAL count reaches `nodes` (program.fs:49,56) or
    max_rounds rounds; every rank of the job must call it with the same arguments.  timer: a
    PhaseTimer (sampled per-phase event timing)."""
    max_batch = _max_batch(engine, max_batch)
    batch = min(batch, max_batch)
    st = engine.sync()
    goal = int(st.round) + max_rounds
    while not st.converged and st.round < goal:
        # gossip's F(k) reports round k-1, so one more exchange than rounds is needed to learn
        # a convergence; rounds issued beyond it are no-ops on the device (gated).
        b = min(batch, goal - int(st.round))
        pieces = getattr(engine, "npieces", 1)
        for _ in range(b):
            ev = timer.events() if timer else None
            if ev:
                ev[0].record()
            if pieces == 1:
                engine.round()
                if ev:
                    ev[1].record()
                transport.exchange(engine)
            else:  # the exchange of piece i overlaps the kernels of piece i+1
                works = []
                for i in range(pieces):
                    engine.round_piece(i)
                    works.append(transport.exchange_piece(engine, i))
                if ev:
                    ev[1].record()  # every piece's kernels enqueued; "exchange": what is left of them
                transport.join(works)
            if ev:
                ev[2].record()
            engine.deliver()
            if ev:
                ev[3].record()
        before = int(st.completed)  # (sync() may refill the same status object)
        st = engine.sync()
        if timer:
            timer.collect()
        batch = _next_batch(batch, max_batch, _nodes(engine), before, int(st.completed))
    return st


def _max_batch(engine, max_batch: int) -> int:
    """The engine's own bound on rounds between syncs, if it has one (HipShard.max_batch)."""
    own = getattr(engine, "max_batch", None)
    return min(max_batch, own) if own else max_batch


def _nodes(engine) -> int:
    return int(engine.layout.nodes)  # HipShard and the oracle's shard engine alike


def _next_batch(batch: int, max_batch: int, nodes: int, before: int, after: int) -> int:
    """Batches double up to max_batch; they start again from 8 rounds when the run enters the
    half-reported phase, where the activity tiers begin (the plan is chosen at every sync, and a
    short run such as full gossip would otherwise reach its end inside one long batch)."""
    if 2 * before < nodes <= 2 * after:
        return min(8, max_batch)
    return min(batch * 2, max_batch)


def run_local(engines, max_rounds: int = 1 << 40, batch: int = 8, max_batch: int = 64):
    """`run` for every shard of a job held in this process (LoopbackTransport)."""
    t = LoopbackTransport()
    max_batch = _max_batch(engines[0], max_batch)
    batch = min(batch, max_batch)
    sts = [e.sync() for e in engines]
    goal = int(sts[0].round) + max_rounds
    while not sts[0].converged and sts[0].round < goal:
        b = min(batch, goal - int(sts[0].round))
        pieces = getattr(engines[0], "npieces", 1)
        for _ in range(b):
            if pieces == 1:
                for e in engines:
                    e.round()
                t.exchange_all(engines)
            else:
                for i in range(pieces):
                    for e in engines:
                        e.round_piece(i)
                    t.piece_done(i)
                    if i:
                        t.exchange_piece_all(engines, i - 1)
                t.exchange_piece_all(engines, pieces - 1)
                t.join()
            for e in engines:
                e.deliver()
        before = int(sts[0].completed)
        sts = [e.sync() for e in engines]
        assert len({(int(s.round), int(s.completed), int(s.converged)) for s in sts}) == 1, "shards disagree"
        batch = _next_batch(batch, max_batch, _nodes(engines[0]), before, int(sts[0].completed))
    return sts

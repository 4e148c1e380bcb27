"""Simulator — the host-side mirror of the reference's program for one run.

/root/reference/program.fs builds a topology of Akka actors (program.fs:150-331), kicks off a
leader and waits for the ParentActor count (program.fs:38-67).  Simulator does the same
through libgossip_hip.so: construction = topology build + InitializeVariables + leader pick,
``run()`` = the message loop until convergence, ``report()`` = the program.fs:51-52 lines.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _abi


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def sizes(n_arg: int, topology: str):
    """(nodes, actors, grid) after program.fs:26-31 / :228-229 rounding."""
    L = _abi.load()
    n, a, g = C.c_int64(), C.c_int64(), C.c_int64()
    _abi.check(L.gp_sizes(n_arg, _abi.TOPOLOGIES[topology], C.byref(n), C.byref(a), C.byref(g)))
    return n.value, a.value, g.value


class Simulator:
    def __init__(self, n_arg: int, topology: str, algorithm: str, *, seed: int = 1, delta: float = 1e-10,
                 gossip_threshold: int = 10, term_init: int = 1, term_limit: int = 3, device: int = 0,
                 kernel_timing: bool = False, generic: bool = False, stream: int | None = None,
                 num_gpus: int = 1, one_device: bool = False, group: bool = False, quiet_waves: bool = False,
                 gossip_tally: bool = False, full_plan: bool = False, tight_tiers: bool = False,
                 tally_fallbacks: bool = False, force_pieces: bool = False, one_round: bool = False,
                 pieces: bool = False):
        """num_gpus > 1: one graph over devices device .. device+num_gpus-1 of this process (the
        library's own RCCL exchange); one_device: all of them on `device` (device-copy exchange);
        group: the multi-GPU engine also for num_gpus = 1; quiet_waves: quiet-wave skipping at any
        graph size (a test hook; it is on by default from 2^20 actors); tally_fallbacks: the receipt
        tally's counted-batch placement and 32-bit receipt escape everywhere (a test hook);
        force_pieces: num_gpus > 1, rounds in 4 pieces at any size (a test hook; the group runs
        them from 2^25 actors per shard); pieces: num_gpus > 1 across devices, exchange in pieces too
        (on by itself with one_device; across devices opt-in until its RCCL path has run on two)."""
        if topology not in _abi.TOPOLOGIES:
            raise ValueError(f"unknown topology {topology!r} (case-sensitive: {list(_abi.TOPOLOGIES)})")
        if algorithm not in _abi.ALGOS:
            raise ValueError("Invalid:Please enter a proper protocol or topology")
        self.lib = _abi.load()
        flags = (_abi.FLAG_KERNEL_TIMING if kernel_timing else 0) | (_abi.FLAG_GENERIC if generic else 0)
        flags |= (_abi.FLAG_ONE_DEVICE if one_device else 0) | (_abi.FLAG_GROUP if group else 0)
        flags |= _abi.FLAG_QUIET_WAVES if quiet_waves else 0
        flags |= _abi.FLAG_GOSSIP_TALLY if gossip_tally else 0
        flags |= _abi.FLAG_TALLY_FALLBACKS if tally_fallbacks else 0
        flags |= _abi.FLAG_FORCE_PIECES if force_pieces else 0
        flags |= _abi.FLAG_PIECES if pieces or force_pieces else 0
        flags |= _abi.FLAG_ONE_ROUND if one_round else 0
        # num_gpus > 1: the exchange plan of the shards (activity tiers; see sharded.HipShard)
        flags |= (_abi.FLAG_FULL_PLAN if full_plan else 0) | (_abi.FLAG_TIGHT_TIERS if tight_tiers else 0)
        if stream is not None:  # an explicit stream, possibly 0 (the null stream)
            flags |= _abi.FLAG_USE_STREAM
        self.cfg = _abi.Config(n_arg, _abi.TOPOLOGIES[topology], _abi.ALGOS[algorithm], seed, delta,
                               gossip_threshold, term_init, term_limit, device, flags, num_gpus, stream)
        self.layout = _abi.Layout()
        h = C.c_void_p()
        _abi.check(self.lib.gp_create(C.byref(self.cfg), C.byref(self.layout), C.byref(h)))
        self.h = h
        self.topology, self.algorithm = topology, algorithm
        self.status = _abi.Status()

    # -- layout ---------------------------------------------------------------------------
    @property
    def nodes(self) -> int:
        return int(self.layout.nodes)

    @property
    def actors(self) -> int:
        return int(self.layout.actors)

    @property
    def leader(self) -> int:
        return int(self.layout.leader)

    # -- running --------------------------------------------------------------------------
    def reset(self):
        _abi.check(self.lib.gp_reset(self.h))
        self.status = _abi.Status()

    def step(self, max_rounds: int = 1 << 40):
        _abi.check(self.lib.gp_step(self.h, max_rounds, C.byref(self.status)))
        return self.status

    run = step

    def report(self) -> str:
        """The reference's final lines (program.fs:51-52) plus the round count."""
        st = self.status
        if not st.converged:
            return f"Not converged after {st.round} rounds ({st.completed} of {self.nodes} reported)"
        return ("-----------------------------------------------------------\n"
                f"Convergence Time: {st.device_ms:f} ms\nRounds: {st.round}")

    # -- read-back ------------------------------------------------------------------------
    def read_gossip(self, first: int = 0, count: int | None = None):
        count = self.actors - first if count is None else count
        cnt = np.zeros(count, np.uint32)
        flags = np.zeros(count, np.uint8)
        _abi.check(self.lib.gp_read_gossip(self.h, first, count, _p(cnt), _p(flags)))
        return cnt, flags

    def read_pushsum(self, first: int = 0, count: int | None = None):
        count = self.actors - first if count is None else count
        S = np.zeros(count, np.float64)
        W = np.zeros(count, np.float64)
        flags = np.zeros(count, np.uint8)
        _abi.check(self.lib.gp_read_pushsum(self.h, first, count, _p(S), _p(W), _p(flags)))
        return S, W, flags

    def read_messages(self, first: int = 0, count: int | None = None):
        count = self.actors - first if count is None else count
        d = np.zeros(count, np.uint32)
        s = np.zeros(count, np.float64)
        w = np.zeros(count, np.float64)
        _abi.check(self.lib.gp_read_messages(self.h, first, count, _p(d), _p(s), _p(w)))
        return d, s, w

    def read_trace(self):
        r = int(self.status.round)
        out = np.zeros(r, np.int64)
        if r:
            _abi.check(self.lib.gp_read_trace(self.h, 0, r, _p(out)))
        return out

    def neighbors(self, v: int):
        cap = 8 if self.topology != "full" else self.nodes
        out = np.zeros(cap, np.uint32)
        d = self.lib.gp_neighbors(self.h, v, _p(out), cap)
        if d < 0:
            _abi.check(d)
        return out[:d]

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

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
